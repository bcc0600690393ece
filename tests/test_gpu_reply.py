"""GPU parity of the 2-ply reply expansion (two_ply.py:114-133): for every
candidate board, the opponent's ordered afterstates for each of the 21
DICE_ROLLS (two_ply.py:10-32), bit for bit against the oracle's movegen
(get_all_possible_moves, generate_all_moves.py:7-90).

The reply launch runs board-major by default (movegen_reply_kernel: the 15
non-doubles rolls of a root in one wave, board_nd_records) and per (board,
roll) job with BGX_REPLY_BM=0; both must give the oracle's lists, and the
engine's records must not depend on the choice.
"""
import numpy as np
import pytest
import torch

import oracle as orc
from test_gpu_parity import _fuzz_positions, _random_positions

pytestmark = pytest.mark.gpu

ROLLS21 = [(a, b) for a in range(1, 7) for b in range(a, 7)]   # DICE_ROLLS order


def _positions():
    pos = _fuzz_positions(77, 24) + _random_positions(5, 1500)
    boards = np.stack([p[0] for p in pos])
    opp = np.array([p[1] for p in pos], np.uint8)
    return boards, opp


def _reply_lists(boards, opp):
    from bgx import ops
    rows, off, cnt = ops.reply_moves(torch.from_numpy(boards).cuda(), torch.from_numpy(opp).cuda())
    torch.cuda.synchronize()
    u8 = ops.unpack(rows).cpu().numpy()
    return u8, off.cpu().numpy(), cnt.cpu().numpy()


@pytest.mark.parametrize("bm,table,dbl,tail", [("1", "0", "1", "4"), ("1", "0", "1", "0"), ("1", "0", "1", "32"),
                                               ("1", "0", "0", "4"), ("0", "0", "0", "4"), ("1", "1", "0", "4")])
def test_reply_moves_vs_oracle(bm, table, dbl, tail, monkeypatch):
    """Self-play and random placements (bar 0-2, borne-off checkers, closed
    boards): every (board, roll) list equals the oracle's, order included, in
    the board-major kernel as shipped (a row's six doubles rolls in one item,
    the last 4/64 of the rows with one item per doubles roll), with every row's
    doubles in one item (BGX_REPLY_DBL_TAIL=0) or half the rows per roll (32),
    with per-roll doubles items only
    (BGX_REPLY_DBL=0), the per-roll kernel and (BGX_MG_TEST_TABLE=1: every root
    through the per-roll hash-table path) the table cross-check."""
    monkeypatch.setenv("BGX_REPLY_BM", bm)
    monkeypatch.setenv("BGX_REPLY_DBL", dbl)
    monkeypatch.setenv("BGX_REPLY_DBL_TAIL", tail)
    monkeypatch.setenv("BGX_MG_TEST_TABLE", table)
    monkeypatch.setenv("BGX_MG_FEW", "0")   # the pool / reply kernels (the engine's large launches)
    boards, opp = _positions()
    u8, off, cnt = _reply_lists(boards, opp)
    kinds = {"bar": 0, "rule": 0, "other": 0}
    for i in range(len(boards)):
        o = int(opp[i])
        home = boards[i, 24 * o + 18:24 * o + 24].sum() if o == 0 else boards[i, 24 * o:24 * o + 6].sum()
        outside = 15 - int(boards[i, 50 + o]) - int(home)
        kinds["bar" if boards[i, 48 + o] else ("rule" if outside >= 3 else "other")] += 1
        for r, (a, b) in enumerate(ROLLS21):
            j = i * 21 + r
            n, res, _ = orc.movegen(boards[i], o, a, b, cap=4096)
            assert cnt[j] == n, (i, a, b, cnt[j], n)
            np.testing.assert_array_equal(u8[off[j]:off[j] + n], res, err_msg=f"board {i} roll {a}-{b}")
    assert min(kinds.values()) > 100, kinds   # every root class is exercised


def test_reply_kernels_agree_on_engine_records(weights_seed0, monkeypatch):
    """Engine 2-ply K=4 and K=all: the records of a run do not depend on the
    reply kernel (board-major, as shipped, vs per-roll). The two kernels
    reserve their output rows differently, so their gap rows (reserved, never
    written, still evaluated by the MLP) differ, but the rows holding records,
    value_rows - gap_rows, are the same count."""
    from bgx import Engine
    from test_gpu_engine import _by_episode, _collect, _same_runs

    def run(bm, k_top):
        monkeypatch.setenv("BGX_REPLY_BM", bm)
        e = Engine(lanes=320 if k_top == 4 else 48, seed=13, ply=2, k_top=k_top)
        e.set_weights(weights_seed0, temperature=1.5, version=1)
        out = _by_episode(*_collect(e, 160 if k_top == 4 else 120, chunk=40))   # games end from ~50 steps
        st = e.stats()
        e.close()
        assert 0 <= st["gap_rows"] < st["value_rows"] // 2, st
        return out, st["value_rows"] - st["gap_rows"]

    for k_top in (4, 0):
        (a, ra), (b, rb) = run("1", k_top), run("0", k_top)
        _same_runs(a, b)
        assert ra == rb, (k_top, ra, rb)
