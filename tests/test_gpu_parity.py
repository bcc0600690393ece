"""GPU parity: libbgx.so kernels vs the reference golden vectors and the CPU oracle.

Bit-exact for move generation (ordered result boards) and encodings; V(s)
within the 1e-5 tolerance of BASELINE.json's north_star.
"""
import hashlib

import numpy as np
import pytest
import torch

from conftest import golden
import oracle as orc

pytestmark = pytest.mark.gpu

V_TOL = 1e-5


@pytest.fixture(scope="module")
def bgx_ops():
    from bgx import ops
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return ops


def _run_movegen(ops, boards, player, dice, cap):
    out, cnt = ops.movegen(torch.from_numpy(np.ascontiguousarray(boards)).cuda(),
                           torch.from_numpy(np.ascontiguousarray(player)).cuda(),
                           torch.from_numpy(np.ascontiguousarray(dice)).cuda(), cap=cap)
    torch.cuda.synchronize()
    return out.cpu().numpy(), cnt.cpu().numpy()


# tier-1 kernel: the balanced pool kernel of large launches ("0") or the
# 16-wave block kernel of small ones ("1"), x the table-free rules for
# doubles / non-doubles (default "0") or the hash-table path for every job ("1")
MG_MODES = [("0", "0"), ("1", "0"), ("0", "1"), ("1", "1")]


@pytest.mark.parametrize("few,table", MG_MODES)
def test_movegen_golden_cases(bgx_ops, few, table, monkeypatch):
    monkeypatch.setenv("BGX_MG_FEW", few)
    monkeypatch.setenv("BGX_MG_TEST_TABLE", table)
    d = golden("movegen_cases.npz")
    out, cnt = _run_movegen(bgx_ops, d["boards"], d["player"], d["dice"], cap=1024)
    for i in range(len(d["boards"])):
        o0, o1 = d["offsets"][i], d["offsets"][i + 1]
        assert cnt[i] == o1 - o0, (i, cnt[i], o1 - o0)
        np.testing.assert_array_equal(out[i, : o1 - o0], d["results"][o0:o1], err_msg=f"case {i}")


@pytest.mark.parametrize("tier", ["2", "3"])
def test_movegen_golden_cases_fallback_tiers(bgx_ops, tier, monkeypatch):
    """Every job forced through the 32 KB LDS tier (2) or the global-memory
    tier (3): the same ordered results as tier 1."""
    monkeypatch.setenv("BGX_MG_TEST_TIER", tier)
    d = golden("movegen_cases.npz")
    out, cnt = _run_movegen(bgx_ops, d["boards"], d["player"], d["dice"], cap=1024)
    for i in range(len(d["boards"])):
        o0, o1 = d["offsets"][i], d["offsets"][i + 1]
        assert cnt[i] == o1 - o0, (tier, i, cnt[i], o1 - o0)
        np.testing.assert_array_equal(out[i, : o1 - o0], d["results"][o0:o1], err_msg=f"tier {tier} case {i}")


def test_movegen_golden_digests(bgx_ops):
    g = golden("movegen_digests.npz")
    n = len(g["boards"])
    for s in range(0, n, 2048):
        e = min(n, s + 2048)
        out, cnt = _run_movegen(bgx_ops, g["boards"][s:e], g["player"][s:e], g["dice"][s:e], cap=512)
        for i in range(e - s):
            assert cnt[i] == g["count"][s + i], s + i
            h = hashlib.sha256(out[i, : cnt[i]].tobytes()).digest()
            assert h == g["sha256"][s + i].tobytes(), s + i


def _fuzz_positions(seed, n_games):
    rng = np.random.default_rng(seed)
    init = golden("movegen_cases.npz")["boards"][0]
    pos = []
    for _ in range(n_games):
        b, pl = init.copy(), int(rng.integers(0, 2))
        for _s in range(300):
            pos.append((b.copy(), pl))
            n, res, _ = orc.movegen(b, pl, int(rng.integers(1, 7)), int(rng.integers(1, 7)))
            if n:
                b = res[int(rng.integers(0, min(n, 500)))].copy()
                if b[50 + pl] >= 15:
                    break
            pl = 1 - pl
    return pos


@pytest.mark.parametrize("few", ["0", "1"])
def test_movegen_fuzz_all_rolls_vs_oracle(bgx_ops, few, monkeypatch):
    monkeypatch.setenv("BGX_MG_FEW", few)
    pos = _fuzz_positions(1234, 40)
    rolls = [(a, b) for a in range(1, 7) for b in range(1, 7)]
    boards = np.stack([p[0] for p in pos for _ in rolls])
    player = np.array([p[1] for p in pos for _ in rolls], np.uint8)
    dice = np.array([r for _ in pos for r in rolls], np.uint8)
    cap = 1024
    for s in range(0, len(boards), 8192):
        e = min(len(boards), s + 8192)
        out, cnt = _run_movegen(bgx_ops, boards[s:e], player[s:e], dice[s:e], cap)
        for i in range(e - s):
            n, res, _ = orc.movegen(boards[s + i], player[s + i], *dice[s + i], cap=cap)
            assert cnt[i] == n, (s + i, cnt[i], n)
            np.testing.assert_array_equal(out[i, :n], res, err_msg=f"job {s + i}")


def _random_positions(seed, n):
    """Checkers dropped uniformly on the points (the two sides on disjoint
    points), a few on the bar or borne off: adjacent blots, stacks and
    reverse chains far more often than self-play reaches them."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        b = np.zeros(52, np.uint8)
        pts = rng.permutation(24)
        k = int(rng.integers(2, 12))
        side = [pts[:k], pts[k:k + int(rng.integers(2, 24 - k))]]
        for pl in (0, 1):
            left = 15
            off = int(rng.choice([0, 0, 0, int(rng.integers(0, 6))]))
            bar = int(rng.choice([0, 0, 0, 0, 1, 2]))
            b[50 + pl], b[48 + pl] = off, bar
            left -= off + bar
            for _c in range(left):
                b[24 * pl + int(rng.choice(side[pl]))] += 1
        out.append((b, int(rng.integers(0, 2))))
    return out


@pytest.mark.parametrize("table", ["0", "1"])
def test_movegen_random_positions_vs_oracle(bgx_ops, table, monkeypatch):
    """Random placements, all 36 rolls; doubles and non-doubles by the
    table-free rules (default) and all through the hash table
    (BGX_MG_TEST_TABLE=1)."""
    monkeypatch.setenv("BGX_MG_TEST_TABLE", table)
    pos = _random_positions(99, 1500)
    rolls = [(a, b) for a in range(1, 7) for b in range(1, 7)]
    boards = np.stack([p[0] for p in pos for _ in rolls])
    player = np.array([p[1] for p in pos for _ in rolls], np.uint8)
    dice = np.array([r for _ in pos for r in rolls], np.uint8)
    cap = 1024
    for s in range(0, len(boards), 8192):
        e = min(len(boards), s + 8192)
        out, cnt = _run_movegen(bgx_ops, boards[s:e], player[s:e], dice[s:e], cap)
        for i in range(e - s):
            n, res, _ = orc.movegen(boards[s + i], player[s + i], *dice[s + i], cap=cap)
            assert cnt[i] == n, (s + i, cnt[i], n)
            np.testing.assert_array_equal(out[i, :n], res, err_msg=f"job {s + i}")


def test_movegen_zero_and_empty(bgx_ops):
    out, cnt = bgx_ops.movegen(torch.zeros((0, 52), dtype=torch.uint8).cuda(),
                               torch.zeros((0,), dtype=torch.uint8).cuda(),
                               torch.zeros((0, 2), dtype=torch.uint8).cuda())
    assert out.shape[0] == 0 and cnt.shape[0] == 0


def test_encode_bit_exact(bgx_ops):
    e = golden("encode.npz")
    b = torch.from_numpy(e["boards"]).cuda()
    p = torch.from_numpy(e["player"]).cuda()
    live = bgx_ops.encode(b, p, 0).cpu().numpy()
    np.testing.assert_array_equal(live.view(np.uint32), e["live"].view(np.uint32))
    n = len(e["interleaved"])
    inter = bgx_ops.encode(b[:n], p[:n], 1).cpu().numpy()
    np.testing.assert_array_equal(inter.view(np.uint32), e["interleaved"].view(np.uint32))


def test_pack_unpack_roundtrip(bgx_ops):
    e = golden("encode.npz")
    b = torch.from_numpy(e["boards"]).cuda()
    p = torch.from_numpy(e["player"]).cuda()
    pk = bgx_ops.pack(b, p)
    np.testing.assert_array_equal(bgx_ops.unpack(pk).cpu().numpy(), e["boards"])
    np.testing.assert_array_equal(bgx_ops.packed_player(pk).cpu().numpy(), e["player"])


@pytest.mark.parametrize("which", ["seed0", "ckpt"])
def test_value_paths_within_tol(bgx_ops, which, weights_seed0, weights_ckpt):
    w = weights_seed0 if which == "seed0" else weights_ckpt
    v = golden("value.npz")
    e = golden("encode.npz")
    ref = v["v_seed0"] if which == "seed0" else v["v_ckpt"]
    net = bgx_ops.Net(w)
    got32 = net.value(torch.from_numpy(v["x"]).cuda()).cpu().numpy()
    assert np.max(np.abs(got32 - ref)) < V_TOL
    gotb = net.value_boards(torch.from_numpy(e["boards"]).cuda(),
                            torch.from_numpy(e["player"]).cuda()).cpu().numpy()
    err = np.max(np.abs(gotb - ref))
    assert err < V_TOL, err
    # and against the fp64 oracle on fresh afterstates
    pos = _fuzz_positions(99, 4)
    boards = np.stack([p[0] for p in pos])
    player = np.array([p[1] for p in pos], np.uint8)
    x = orc.encode_many(boards, player)
    want = orc.value(w, x)
    got = net.value_boards(torch.from_numpy(boards).cuda(), torch.from_numpy(player).cuda()).cpu().numpy()
    assert np.max(np.abs(got - want)) < V_TOL


def test_stateless_ops_reject_out_of_domain_inputs(bgx_ops, weights_seed0):
    """The device check (include/bgx.h BGX_BADF_*) of every stateless entry
    point: each rule rejects with BGX_E_ARG before any output is written, the
    device flags equal the host rule's, and legal inputs pass."""
    from bgx import BgxError
    from test_abi import _host_check, domain_cases
    cases = domain_cases()
    boards = np.stack([c[1] for c in cases])
    players = np.array([c[2] for c in cases], np.uint8)
    dice = np.array([c[3] for c in cases], np.uint8)
    # device flags == host flags, per case and for the whole batch
    for k in range(len(cases)):
        got = bgx_ops.check_boards(torch.from_numpy(boards[k:k + 1]).cuda(),
                                   torch.from_numpy(players[k:k + 1]).cuda(),
                                   torch.from_numpy(dice[k:k + 1]).cuda())
        assert got == _host_check(boards[k:k + 1], players[k:k + 1], dice[k:k + 1]), cases[k][0]
    assert bgx_ops.check_boards(torch.from_numpy(boards).cuda(), torch.from_numpy(players).cuda(),
                                torch.from_numpy(dice).cuda()) == (31, 3)
    net = bgx_ops.Net(weights_seed0)
    for k, (name, b, p, d, want) in enumerate(cases):
        bb = torch.from_numpy(np.stack([cases[0][1], b])).cuda()     # a legal row first
        pp = torch.tensor([0, min(p, 255)], dtype=torch.uint8).cuda()
        dd = torch.tensor([[3, 1], list(d)], dtype=torch.uint8).cuda()
        for fn, bad in (
                (lambda: bgx_ops.movegen(bb, pp, dd, cap=64), want),
                (lambda: bgx_ops.encode(bb, pp), want & ~8),
                (lambda: net.value_boards(bb, pp), want & ~8),
                (lambda: net.two_ply(bb, pp), want & ~8)):
            if bad:
                with pytest.raises(BgxError, match="outside the board domain"):
                    fn()
            else:
                fn()
    torch.cuda.synchronize()


def test_stateless_ops_thread_safe_scratch(bgx_ops):
    """Concurrent bgx_movegen calls from several host threads on their own
    streams (each call leases its own overflow counter / workspace) give the
    single-threaded results."""
    import threading
    g = golden("movegen_cases.npz")
    boards, player, dice = g["boards"][:400], g["player"][:400], g["dice"][:400]
    want_out, want_cnt = _run_movegen(bgx_ops, boards, player, dice, 64)
    errs, outs = [], {}

    def work(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for rep in range(6):
                    o, c = bgx_ops.movegen(torch.from_numpy(boards).cuda(), torch.from_numpy(player).cuda(),
                                           torch.from_numpy(dice).cuda(), cap=64, stream=s)
                    s.synchronize()
                    outs[(t, rep)] = (o.cpu().numpy(), c.cpu().numpy())
        except Exception as ex:   # noqa: BLE001
            errs.append(ex)

    th = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errs, errs
    assert len(outs) == 24
    for o, c in outs.values():
        np.testing.assert_array_equal(c, want_cnt)
        for i in range(len(c)):
            k = min(int(c[i]), 64)
            np.testing.assert_array_equal(o[i, :k], want_out[i, :k])
