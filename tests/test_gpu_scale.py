"""Parity at the benchmarked scale and run-to-run reproducibility.

* The bench's exact 1-ply shape (bench.py run_engine): Engine(8,192 lanes,
  balance=True) -- the FL = 32 fused kernel, one 32-lane group per CU, the
  balanced lane-step budget, the tier-1 expansion carried across launches, the
  in-kernel harvest into three rotating slots -- driven as bench.py drives
  it: 300 desync steps, then two 300-step launches, each harvest queued
  behind its launch (harvest_enqueue) and fetched while the next launch runs.
  Every header of every harvest is checked for the episode bookkeeping
  (each lane's episodes 0, 1, 2, ... exactly once, contiguous first records,
  lengths, terminal flags), and a seeded random sample of whole episodes
  holding >= 20,000 records is replayed transition by transition through the
  oracle (test_gpu_engine._check_transitions: afterstate, V(s) / V(a),
  reward, done, win type, shaping, observations). Reference loop:
  src/multi/worker.py:101-162 over backgammon_env.py:130-308.
* 2-ply K = all at 4,096 lanes (configs[2]'s lane count), greedy: >= 2,000
  sampled decisions equal the oracle's argmax of 1.0 * V - 0.9 * W over every
  candidate (two_ply.py:44-150).
* 2-ply at the bench's own 8,192-lane shape (round 6): K = all greedy, >= 2,000
  decisions equal the oracle's argmax, and one step peeked between two
  bgx_engine_peek calls gives, for >= 500 lanes, the oracle's candidate boards
  (bit-exact), V within 1e-5 and the W of every candidate (the DICE_ROLLS-
  weighted top-5 reply means the step computed) within 1e-5 of the oracle's
  two_ply_response; K = 4 (the bench's sampling leg): the engine's top 4 by V
  and each one's W, 500 lanes. The same peeked check at configs[2]'s 4,096
  lanes for both legs bench.py times there (K = 4 and K = all).
* The same seed twice in one process gives identical records for 2-ply
  reference-sampled (reply_sample = 50, two_ply.py:119-121) and K = all
  (DESIGN.md section 4 argues why no kernel reads a reply row outside its
  job's range; this is the run-level check).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle as orc
from test_gpu_engine import _by_episode, _check_transitions, _collect, _same_runs

pytestmark = pytest.mark.gpu
V_TOL = 1e-5


def _engine(weights, **kw):
    from bgx import Engine
    e = Engine(**kw)
    e.set_weights(weights, temperature=1.5, version=1)
    return e


def _bench_run(e, n, chunk, out):
    """bench.py run_engine's run(): launch, queue its harvest, fetch the
    previous one while this launch runs; harvests copied to host as fetched."""
    left, pending = n, None

    def take(t):
        h = e.harvest_fetch(t)
        out.append((h.headers.cpu().numpy().view(np.uint32).copy(), h.records.cpu().numpy().view(np.uint32).copy()))

    while left > 0:
        k = min(chunk, left)
        e.step(k)
        t = e.harvest_enqueue()
        if pending is not None:
            take(pending)
        pending = t
        left -= k
    take(pending)


def _check_headers(harvests, lanes, max_steps=300):
    """Episode bookkeeping over every harvest: lanes in range, each lane's
    episode numbers 0, 1, 2, ... exactly once and in order across harvests,
    each episode's records contiguous after its predecessor's, lengths and
    terminal flags consistent. Returns the number of episodes."""
    from bgx.records import fields
    nxt_ep = np.zeros(lanes, np.int64)
    nxt_rec = np.zeros(lanes, np.int64)
    n_eps = 0
    for hdr, rec in harvests:
        assert rec.shape[0] == int(hdr[:, 3].astype(np.int64).sum())
        f = fields(rec)
        o = 0
        for row in hdr:
            lane, ep, first, n, steps = (int(x) for x in row[:5])
            assert 0 <= lane < lanes
            assert ep == nxt_ep[lane], (lane, ep, nxt_ep[lane])
            assert first == nxt_rec[lane], (lane, ep, first, nxt_rec[lane])
            nxt_ep[lane] += 1
            nxt_rec[lane] += n
            assert 1 <= n <= steps <= max_steps
            st = f["step"][o:o + n]
            assert np.all(np.diff(st) >= 1) and st[0] >= 0 and st[-1] < steps
            done = f["done"][o:o + n]
            assert not done[:-1].any()
            if steps < max_steps:   # a game that ended before the step cap ended on a win
                assert done[-1] and st[-1] == steps - 1 and f["win_type"][o + n - 1] > 0
                assert int(row[5]) & 0xFF == int(f["win_type"][o + n - 1])
            assert not f["win_type"][o:o + n - 1].any()
            o += n
            n_eps += 1
    return n_eps


def _subset(hdr, rec, pick):
    """Headers `pick` (indices into hdr) and their records, concatenated."""
    offs = np.concatenate([[0], np.cumsum(hdr[:, 3].astype(np.int64))])
    sub = hdr[pick]
    parts = [rec[offs[i]:offs[i + 1]] for i in pick]
    return sub, np.concatenate(parts) if parts else rec[:0]


def test_bench_shape_1ply_matches_oracle(weights_seed0):
    import torch
    from bgx.episodes import decode_records
    lanes, chunk = 8192, 300
    e = _engine(weights_seed0, lanes=lanes, seed=0, ply=1, balance=True)
    assert e.fused
    harvests = []
    _bench_run(e, 300, chunk, harvests)        # bench.py --desync-steps
    s0 = e.stats()
    _bench_run(e, 600, chunk, harvests)        # two 300-step launches, pipelined harvests
    s1 = e.stats()
    e.close()
    groups = lanes // 32
    done = s1["env_steps"] - s0["env_steps"]
    # the budget, plus less than one 32-lane workgroup-step per workgroup and launch
    assert lanes * 600 <= done < lanes * 600 + 2 * groups * 32, done
    n_eps = _check_headers(harvests, lanes)
    assert n_eps > 20000
    # a seeded random sample of whole episodes, >= 20,000 records, through the oracle
    rng = np.random.default_rng(2026)
    checked = 0
    for hdr, rec in harvests:
        order = rng.permutation(hdr.shape[0])
        lens = hdr[order, 3].astype(np.int64)
        take = order[:int(np.searchsorted(np.cumsum(lens), 7000)) + 1]
        sub_h, sub_r = _subset(hdr, rec, np.sort(take))
        d = decode_records(sub_h, torch.from_numpy(sub_r.view(np.int32)).cuda())
        checked += _check_transitions(weights_seed0, [sub_h], [d], 1)
    assert checked >= 20000, checked


def _kall_scores(w, board, mover, d0, d1):
    """two_ply.py:44-90 with every candidate: 1.0 * V - 0.9 * W (oracle, fp64)."""
    cnt, res, _ = orc.movegen(board, mover, d0, d1)
    m = min(cnt, 500)
    v = orc.value(w, orc.encode_many(res[:m], [mover] * m))
    W = np.array([orc.two_ply_response(w, res[c], 1 - mover) for c in range(m)])
    return 1.0 * v - 0.9 * W


def test_kall_4096_lanes_greedy_is_oracle_argmax(weights_seed0):
    from bgx.episodes import decode_records
    lanes = 4096
    e = _engine(weights_seed0, lanes=lanes, seed=19, ply=2, k_top=0, greedy=True)
    e.step(150)
    h = e.harvest()
    hdr = h.headers.cpu().numpy().view(np.uint32)
    d = decode_records(hdr, h.records)
    e.close()
    m = d["action"].shape[0]
    assert m > 20000
    rng = np.random.default_rng(7)
    ks = rng.choice(m, 2000, replace=False)

    def one(k):
        s = _kall_scores(weights_seed0, d["before"][k], int(d["mover"][k]), *d["dice"][k])
        a = int(d["action"][k])
        return a, float(s[a]), float(s.max()), len(s)

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:   # ctypes drops the GIL
        res = list(ex.map(one, ks))
    for k, (a, sa, smax, n) in zip(ks, res):
        assert 0 <= a < n
        assert sa >= smax - 2 * V_TOL, (int(k), a, sa, smax)
    assert len(res) == 2000


# two_ply.py:10-32 DICE_ROLLS order; a double has probability 1/36, the others 2/36
ROLLS = [(a, b) for a in range(1, 7) for b in range(a, 7)]
ROLL_P = np.array([1.0 / 36 if a == b else 2.0 / 36 for a, b in ROLLS])


def _unpack(w):
    """packed rows uint32 [n, 8] -> uint8 [n, 52] (bgx_device.h packed_to_u8)"""
    w = np.asarray(w, np.uint32).reshape(-1, 8)
    out = np.zeros((w.shape[0], 52), np.uint8)
    for k in range(6):
        for q in range(8):
            out[:, 8 * k + q] = (w[:, k] >> (4 * q)) & 15
    for i in range(4):
        out[:, 48 + i] = (w[:, 6] >> (4 * i)) & 15
    return out


def _peek_step(e):
    """One engine step between two peeks: the lanes' positions before it, and
    the candidates, V and per-(candidate, roll) top-5 reply means it computed."""
    before = {k: e.peek(k) for k in ("lane_rows", "player", "dice")}
    e.step(1)
    after = {k: e.peek(k) for k in ("cand_off", "cand_cnt", "cand_rows", "values", "job_val")}
    if e.cfg.k_top == 4:
        after["sel"] = e.peek("sel")
    return before, after


def _check_lane_w(w, lanes, before, after, i):
    """Lane i of a peeked 2-ply step against the oracle: its candidate boards
    in the reference's order (bit-exact), V(candidate) within 1e-5, and W of
    every candidate the step scored (K = all: every one; K = 4: the top 4 by V)
    as the DICE_ROLLS-weighted top-5 means, within 1e-5 of the oracle's
    two_ply_response (two_ply.py:93-150). Returns the number of W compared."""
    board = _unpack(before["lane_rows"][i])[0]
    mover = int(before["player"][i])
    d0, d1 = (int(x) for x in before["dice"][i])
    cnt, res, _ = orc.movegen(board, mover, d0, d1)
    assert int(after["cand_cnt"][i]) == cnt, (i, int(after["cand_cnt"][i]), cnt)
    m = min(cnt, 500)
    if m == 0:
        return 0
    off = int(after["cand_off"][i])
    got = _unpack(after["cand_rows"][off:off + m])
    assert np.array_equal(got, res[:m]), i
    v = orc.value(w, orc.encode_many(res[:m], [mover] * m))
    gv = after["values"][lanes + off:lanes + off + m].astype(np.float64)
    assert np.abs(gv - v).max() < V_TOL, (i, float(np.abs(gv - v).max()))
    if "sel" in after:
        sel = after["sel"][i]
        if sel[0] < 0:
            assert m < 4
            return 0
        cand = [int(s) - lanes - off for s in sel]
        rest = np.delete(v, cand)
        assert len(set(cand)) == 4 and (rest.size == 0 or v[cand].min() >= rest.max() - V_TOL), (i, cand)
        jv = after["job_val"].reshape(-1, 21)[4 * i:4 * i + 4]
    else:
        cand = list(range(m))
        jv = after["job_val"].reshape(-1, 21)[off:off + m]
    n = 0
    for c, row in zip(cand, jv):
        assert 0 <= c < m
        W_eng = float(np.dot(row.astype(np.float64), ROLL_P))
        W_orc = orc.two_ply_response(w, res[c], 1 - mover)
        assert abs(W_eng - W_orc) < V_TOL, (i, c, W_eng, W_orc)
        n += 1
    return n


def test_kall_8192_lanes_w_and_greedy_argmax(weights_seed0):
    """2-ply K = all at the bench's 8,192-lane shape (bench.py's K = all leg:
    the same grid, reply row chunks and refills), greedy. (1) One step between
    two peeks (bgx_engine_peek): for >= 500 lanes the step's candidate boards
    equal the oracle's movegen, their V is within 1e-5, and W of every
    candidate -- the DICE_ROLLS-weighted means of the engine's per-(candidate,
    roll) top-5 reply values -- is within 1e-5 of the oracle's
    two_ply_response (two_ply.py:93-150). (2) >= 2,000 sampled decisions of
    the following steps equal the oracle's argmax of 1.0 * V - 0.9 * W
    (two_ply.py:44-90)."""
    from bgx.episodes import decode_records
    lanes = 8192
    e = _engine(weights_seed0, lanes=lanes, seed=37, ply=2, k_top=0, greedy=True)
    e.step(100)                 # lanes spread over their games
    e.harvest()
    before, after = _peek_step(e)
    e.step(60)
    h = e.harvest()
    hdr = h.headers.cpu().numpy().view(np.uint32)
    d = decode_records(hdr, h.records)
    e.close()
    rng = np.random.default_rng(13)
    movers = [i for i in rng.permutation(lanes) if int(after["cand_cnt"][i]) > 0][:600]
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:   # ctypes drops the GIL
        nw = list(ex.map(lambda i: _check_lane_w(weights_seed0, lanes, before, after, i), movers))
    assert len(movers) == 600 and sum(nw) >= 5000, (len(movers), sum(nw))

    m = d["action"].shape[0]
    assert m > 20000
    ks = rng.choice(m, 2000, replace=False)

    def one(k):
        s = _kall_scores(weights_seed0, d["before"][k], int(d["mover"][k]), *d["dice"][k])
        a = int(d["action"][k])
        return a, float(s[a]), float(s.max()), len(s)

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        res = list(ex.map(one, ks))
    for k, (a, sa, smax, n) in zip(ks, res):
        assert 0 <= a < n
        assert sa >= smax - 2 * V_TOL, (int(k), a, sa, smax)


def test_k4_8192_lanes_w(weights_seed0):
    """2-ply K = 4 at 8,192 lanes (bench.py's K = 4 leg, sampling as the bench
    runs it): one peeked step, >= 500 lanes with >= 4 moves -- the engine's
    top 4 by V and each one's W within 1e-5 of the oracle's."""
    lanes = 8192
    e = _engine(weights_seed0, lanes=lanes, seed=43, ply=2, k_top=4)
    e.step(100)
    e.harvest()
    before, after = _peek_step(e)
    e.close()
    rng = np.random.default_rng(17)
    movers = [i for i in rng.permutation(lanes) if int(after["cand_cnt"][i]) >= 4][:500]
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        nw = list(ex.map(lambda i: _check_lane_w(weights_seed0, lanes, before, after, i), movers))
    assert len(movers) == 500 and sum(nw) == 2000


@pytest.mark.parametrize("k_top", [4, 0])
def test_configs2_4096_lanes_w(weights_seed0, k_top):
    """configs[2]'s own shape (4,096 lanes, bench.py's configs2_4096_lanes
    legs; a grid of half the 8,192-lane one per launch): one peeked step, the
    candidates, V and every scored candidate's W against the oracle (K = 4:
    300 lanes with >= 4 moves, sampling; K = all: 250 lanes, greedy)."""
    lanes = 4096
    e = _engine(weights_seed0, lanes=lanes, seed=53 + k_top, ply=2, k_top=k_top, greedy=k_top == 0)
    e.step(100)
    e.harvest()
    before, after = _peek_step(e)
    e.close()
    rng = np.random.default_rng(23)
    need, n_lanes = (4, 300) if k_top == 4 else (1, 250)
    movers = [i for i in rng.permutation(lanes) if int(after["cand_cnt"][i]) >= need][:n_lanes]
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        nw = list(ex.map(lambda i: _check_lane_w(weights_seed0, lanes, before, after, i), movers))
    assert len(movers) == n_lanes
    assert sum(nw) == 4 * n_lanes if k_top == 4 else sum(nw) >= 2000, sum(nw)


@pytest.mark.parametrize("k_top,sample", [(4, 50), (0, 0)])
def test_2ply_same_seed_same_records(weights_seed0, k_top, sample):
    """Two engines with the same seed, one after the other in one process:
    identical episodes and records (2-ply reference-sampled and K = all)."""
    runs = []
    for _ in range(2):
        e = _engine(weights_seed0, lanes=256, seed=41, ply=2, k_top=k_top, reply_sample=sample)
        runs.append(_by_episode(*_collect(e, 90 if k_top else 60, chunk=30)))
        e.close()
    _same_runs(*runs)


def test_k4_8192_lanes_greedy_is_oracle_argmax(weights_seed0):
    """2-ply K = 4 at the 8,192-lane shard (configs[4]'s per-GPU shape, the
    bench's 2-ply leg), greedy, after >= 100 steps: >= 2,000 sampled decisions
    equal the oracle's argmax of 1.0 * V - 0.9 * W over the top 4 by V
    (two_ply.py:44-90, 153-193; fewer than 4 moves: the 1-ply argmax)."""
    from bgx.episodes import decode_records
    from test_gpu_replay import _two_ply_scores
    e = _engine(weights_seed0, lanes=8192, seed=23, ply=2, k_top=4, greedy=True)
    e.step(100)
    e.harvest()
    e.step(40)
    h = e.harvest()
    hdr = h.headers.cpu().numpy().view(np.uint32)
    d = decode_records(hdr, h.records)
    e.close()
    m = d["action"].shape[0]
    assert m > 10000
    rng = np.random.default_rng(11)
    ks = rng.choice(m, 3200, replace=False)   # ~74 % have >= 4 moves (2-ply); the rest the 1-ply argmax

    def one(k):
        a = int(d["action"][k])
        r = _two_ply_scores(weights_seed0, d["before"][k], int(d["mover"][k]), *d["dice"][k], 4)
        if r[0] is None:
            v = r[1]
            return "1ply", v[a] >= v.max() - V_TOL, (a, float(v[a]), float(v.max()))
        cand, score, v = r
        if a not in set(cand.tolist()):   # only a V tie at the top-4 boundary moves a candidate in or out
            return "tie", abs(v[a] - v[cand[-1]]) < V_TOL, (a, float(v[a]), float(v[cand[-1]]))
        return "2ply", score[list(cand).index(a)] >= score.max() - 2 * V_TOL, (a, score.tolist())

    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        res = list(ex.map(one, ks))
    for k, (kind, ok, info) in zip(ks, res):
        assert ok, (int(k), kind, info)
    assert sum(kind == "2ply" for kind, _, _ in res) >= 2000


def test_k4_8192_lanes_sampling_transitions(weights_seed0):
    """2-ply K = 4 sampling at 8,192 lanes: a seeded sample of whole episodes
    holding >= 5,000 records replayed through the oracle transition by
    transition (afterstate, V(s) / V(a), rewards, observations; the chosen
    move is one of the legal ones)."""
    import torch
    from bgx.episodes import decode_records
    e = _engine(weights_seed0, lanes=8192, seed=29, ply=2, k_top=4)
    e.step(150)
    h = e.harvest()
    hdr = h.headers.cpu().numpy().view(np.uint32)
    rec = h.records.cpu().numpy().view(np.uint32)
    e.close()
    assert _check_headers([(hdr, rec)], 8192) > 1000
    rng = np.random.default_rng(5)
    order = rng.permutation(hdr.shape[0])
    lens = hdr[order, 3].astype(np.int64)
    take = order[:int(np.searchsorted(np.cumsum(lens), 5000)) + 1]
    sub_h, sub_r = _subset(hdr, rec, np.sort(take))
    d = decode_records(sub_h, torch.from_numpy(sub_r.view(np.int32)).cuda())
    assert _check_transitions(weights_seed0, [sub_h], [d], 2) >= 5000


@pytest.mark.parametrize("k_top", [4, 0])
def test_reply_delta_opt_in_w(weights_seed0, k_top, monkeypatch):
    """The opt-in reply MLP by difference from the root (BGX_REPLY_DELTA=1,
    mlp_kernel_delta; measured slower and not the default): one
    peeked step of a 2,048-lane engine, W of >= 150 lanes' candidates within
    1e-5 of the oracle's two_ply_response (K = 4: the chosen rows' own root
    launch, roots by slot; K = all: the root launch's accumulators)."""
    monkeypatch.setenv("BGX_REPLY_DELTA", "1")
    lanes = 2048
    e = _engine(weights_seed0, lanes=lanes, seed=47, ply=2, k_top=k_top)
    e.step(60)
    e.harvest()
    before, after = _peek_step(e)
    e.close()
    rng = np.random.default_rng(19)
    need = 4 if k_top == 4 else 1
    movers = [i for i in rng.permutation(lanes) if int(after["cand_cnt"][i]) >= need][:150]
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        nw = list(ex.map(lambda i: _check_lane_w(weights_seed0, lanes, before, after, i), movers))
    assert len(movers) == 150 and sum(nw) >= 600
