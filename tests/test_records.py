"""The harvest wire format (bgx/records.py, include/bgx.h bgx_harvest): 48-B
records whose after-board is the next record's before-board or the header's
final board, with the next_observation indicator rule of
backgammon_env.py:196-218 (the winner at a terminal step, else the other
player). CPU only."""
import numpy as np

from bgx.records import EP_WORDS, REC_WORDS, fields, pack_record, packed_before_after


def _board(seed):
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 2**31, 7).astype(np.uint32)
    w[6] &= 0xFFFF
    return w


def test_fields_round_trip():
    r = pack_record(_board(1), 1, 0.25, -0.5, 0.3, 499, 4500, 299, (6, 5), 0, 1, 1, 0)
    f = fields(r[None])
    assert f["action"][0] == 499 and f["n_moves"][0] == 4095 and f["step"][0] == 299   # n_moves saturates
    assert tuple(f["dice"][0]) == (6, 5) and f["mover"][0] == 1 and not f["done"][0]
    assert f["close_out"][0] and f["prime"][0] and f["win_type"][0] == 0
    assert f["v_s"][0] == np.float32(0.25) and f["v_a"][0] == np.float32(-0.5) and f["reward"][0] == np.float32(0.3)


def test_after_boards_and_indicators():
    # episode A: 3 records, ends in a win by player 0; episode B: 2 records, truncated
    boards = [_board(s) for s in range(7)]
    recs = [pack_record(boards[0], 0, 0, 0, 0, 1, 5, 0, (3, 1), 0, 0, 0, 0),
            pack_record(boards[1], 1, 0, 0, 0, 2, 5, 1, (4, 2), 0, 0, 0, 0),
            pack_record(boards[2], 0, 0, 0, 1.0, 0, 3, 4, (6, 6), 1, 0, 0, 1),   # two passes before
            pack_record(boards[4], 1, 0, 0, 0, 0, 9, 0, (2, 1), 0, 0, 0, 0),
            pack_record(boards[5], 0, 0, 0, 0, 3, 9, 1, (5, 2), 0, 0, 0, 0)]
    hdr = np.zeros((2, EP_WORDS), np.uint32)
    hdr[0, 3], hdr[0, 6:13] = 3, boards[3]
    hdr[1, 3], hdr[1, 6:13] = 2, boards[6]
    before, after = packed_before_after(hdr, np.stack(recs))
    assert before.shape == (5, 8) and after.shape == (5, 8)
    flag = lambda w: int(w[6] >> 16)   # noqa: E731
    for k, (b, m) in enumerate([(0, 0), (1, 1), (2, 0), (4, 1), (5, 0)]):
        np.testing.assert_array_equal(before[k, :6], boards[b][:6])
        assert before[k, 6] & 0xFFFF == boards[b][6] & 0xFFFF and flag(before[k]) == m
    want_after = [(1, 1), (2, 0), (3, 0), (5, 0), (6, 1)]   # (board, indicator): terminal keeps the winner
    for k, (b, m) in enumerate(want_after):
        np.testing.assert_array_equal(after[k, :6], boards[b][:6])
        assert after[k, 6] & 0xFFFF == boards[b][6] & 0xFFFF and flag(after[k]) == m, k
    assert REC_WORDS * 4 == 48 and EP_WORDS * 4 == 64
