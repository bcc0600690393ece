"""GPU engine vs the reference's own env trajectories, shard invariance and
2-ply decisions against the oracle.

* Replay: tests/golden/env_traj.npz holds greedy
  episodes that tools/gen_golden.py played with the reference's functions in
  the order BackgammonEnv.reset / step run them (backgammon_env.py:92-221,
  worker.py:101-162), with every np.random.randint die recorded, under the
  seed-0 weights and the shipped 2.1M checkpoint; they include close-outs,
  primes, repeats of either after the reward was given, gammons, backgammons
  and consecutive passes (test_oracle_golden.py counts them). The engine
  replays them with those dice scripted (bgx_engine_set_dice) and greedy
  play, and every decision must match: board before and after, mover through
  pass turns, dice, move count, action, V(s) / V(a) (1e-5), reward, done, win
  type, shaping flags, and the 198-d observation / next_observation (the
  winner's indicator at the terminal step) bit for bit.
* Shard invariance: lanes are keyed by their global id, so
  Engine(L, lane_base=0) and Engine(L, lane_base=L) produce exactly the
  episodes of lanes 0..2L-1 of one Engine(2L) (main.py:86-91 splits the work
  over workers; here over GPUs).
* 2-ply (two_ply.py:44-150 + the worker hook 153-193): greedy picks equal the
  argmax of alpha * V - beta * W computed by the oracle, for K = 4 and for
  every candidate (K = all); sampled K = 4 picks follow softmax(score / T).
"""
import numpy as np
import pytest
import torch

from conftest import golden
import oracle as orc

pytestmark = pytest.mark.gpu
V_TOL = 1e-5


def _engine(weights, **kw):
    from bgx import Engine
    e = Engine(**kw)
    e.set_weights(weights, temperature=1.5, version=1)
    return e


def _episodes(e, steps, chunk=100):
    """{(lane, episode no.): (header row, decoded record fields)}"""
    from bgx.episodes import decode_records
    out = {}
    done = 0
    while done < steps:
        k = min(chunk, steps - done)
        e.step(k)
        h = e.harvest()
        hdr = h.headers.cpu().numpy().view(np.uint32)
        d = decode_records(hdr, h.records)
        o = 0
        for row in hdr:
            n = int(row[3])
            out[(int(row[0]), int(row[1]))] = (row.copy(), {f: v[o:o + n] for f, v in d.items()})
            o += n
        done += k
    e.sync()
    return out


@pytest.mark.parametrize("wset", [0, 1])
@pytest.mark.parametrize("fused", [False, True])
def test_replay_reference_trajectories(weights_seed0, weights_ckpt, fused, wset):
    t = golden("env_traj.npz")
    eps = t["episodes"][t["weight_set"] == wset]
    n = len(eps)
    # after its episode a lane keeps playing (new games on 1-2 rolls): two
    # draws per env step for the rest of the 300 steps, plus the resets
    width = int(max(eps[:, 1])) + 2 * 300 + 64
    dice = np.tile(np.array([1, 2], np.uint8), (n, width // 2 + 1))[:, :width].copy()
    for i, (d0, dn, _s0, _sn) in enumerate(eps):
        dice[i, :dn] = t["dice"][d0:d0 + dn]
    e = _engine(weights_seed0 if wset == 0 else weights_ckpt, lanes=n, seed=0, ply=1, greedy=True, fused=fused)
    e.set_dice(dice)
    got = _episodes(e, 300, chunk=150)
    e.close()
    checked = 0
    for i, (_d0, _dn, s0, sn) in enumerate(eps):
        hdr, d = got[(i, 0)]
        rows = np.arange(s0, s0 + sn)
        dec = rows[t["kind"][rows] == 0]
        assert int(hdr[3]) == len(dec), i                 # one Experience per decision
        assert int(hdr[4]) == sn, i                       # env steps, passes included
        step_of = {int(r): k for k, r in enumerate(rows)}
        for k, r in enumerate(dec):
            r = int(r)
            mover = int(t["player"][r])
            np.testing.assert_array_equal(d["before"][k], t["board"][r], err_msg=f"ep {i} row {r}")
            np.testing.assert_array_equal(d["after"][k], t["after"][r], err_msg=f"ep {i} row {r}")
            assert int(d["mover"][k]) == mover
            assert int(d["step"][k]) == step_of[r]
            assert tuple(d["dice"][k]) == tuple(int(x) for x in t["roll"][r])
            assert int(d["n_moves"][k]) == int(t["full_moves"][r])
            assert int(d["action"][k]) == int(t["action"][r]), (i, r)
            assert abs(float(d["v_s"][k]) - float(t["v_obs"][r])) < V_TOL
            assert abs(float(d["v_a"][k]) - float(t["v_act"][r])) < V_TOL
            assert d["reward"][k] == np.float32(t["reward"][r])
            assert bool(d["done"][k]) == bool(t["done"][r])
            assert int(d["win_type"][k]) == int(t["win_type"][r])
            assert bool(d["close_out"][k]) == bool(t["close_out"][r])
            assert bool(d["prime"][k]) == bool(t["prime"][r])
            np.testing.assert_array_equal(d["obs"][k], orc.encode(t["board"][r], mover))
            nxt = mover if t["done"][r] else 1 - mover
            np.testing.assert_array_equal(d["next_obs"][k], orc.encode(t["after"][r], nxt))
            checked += 1
        last = int(rows[-1])
        if t["done"][last]:
            assert int(hdr[5]) & 0xFF == int(t["win_type"][last])
            assert (int(hdr[5]) >> 8) & 0xFF == int(t["player"][last])
    rows = np.concatenate([np.arange(s0, s0 + sn) for (_d0, _dn, s0, sn) in eps])
    assert checked == int((t["kind"][rows] == 0).sum())


def test_scripted_dice_need_greedy_and_report_exhaustion(weights_seed0):
    from bgx import BgxError
    e = _engine(weights_seed0, lanes=4, seed=0, ply=1)
    with pytest.raises(BgxError):
        e.set_dice(np.ones((4, 8), np.uint8))     # sampling lanes cannot take scripted dice
    e.close()
    e = _engine(weights_seed0, lanes=4, seed=0, ply=1, greedy=True, fused=False)
    e.set_dice(np.tile(np.array([3, 1, 4, 2], np.uint8), (4, 2)))   # reset + 2 rolls per lane
    e.step(5)
    with pytest.raises(BgxError, match="flags"):
        e.sync()
    e.close()


@pytest.mark.parametrize("ply,k_top,fused", [(1, 4, True), (1, 4, False), (2, 4, False)])
def test_shard_invariance(weights_seed0, ply, k_top, fused):
    """Two engines over lane blocks [0, L) and [L, 2L) == one engine of 2L lanes."""
    L, steps = (96, 150) if ply == 1 else (32, 160)
    kw = dict(seed=7, ply=ply, k_top=k_top, fused=fused)
    whole = _episodes(_engine(weights_seed0, lanes=2 * L, **kw), steps, chunk=80)
    parts = {}
    for base in (0, L):
        parts.update(_episodes(_engine(weights_seed0, lanes=L, lane_base=base, **kw), steps, chunk=80))
    assert len(whole) > 10 and whole.keys() == parts.keys()
    for key in whole:
        np.testing.assert_array_equal(whole[key][0][1:], parts[key][0][1:], err_msg=str(key))   # header (not 'first')
        for f in whole[key][1]:
            np.testing.assert_array_equal(whole[key][1][f], parts[key][1][f], err_msg=f"{key} {f}")


def _two_ply_scores(w, board, mover, d0, d1, k_top):
    """(candidate indices, scores): two_ply.py:44-90 on the oracle; K = 4 takes
    the top 4 by V (torch.topk: ties to the lower index), K = all every
    candidate; None when K = 4 and fewer than 4 moves (1-ply fallback)."""
    cnt, res, _ = orc.movegen(board, mover, d0, d1)
    m = min(cnt, 500)
    v = orc.value(w, orc.encode_many(res[:m], [mover] * m))
    if k_top == 4 and m < 4:
        return None, v
    cand = np.argsort(-v, kind="stable")[:4] if k_top == 4 else np.arange(m)
    W = np.array([orc.two_ply_response(w, res[c], 1 - mover) for c in cand])
    return cand, 1.0 * v[cand] - 0.9 * W, v


@pytest.mark.parametrize("k_top,lanes,steps,check", [(4, 48, 150, 700), (0, 16, 150, 120)])
def test_engine_2ply_greedy_is_oracle_argmax(weights_seed0, k_top, lanes, steps, check):
    """The first `check` decisions of finished greedy games (the oracle's
    2-ply costs ~8 ms per candidate in C)."""
    e = _engine(weights_seed0, lanes=lanes, seed=3, ply=2, k_top=k_top, greedy=True)
    got = _episodes(e, steps, chunk=steps)
    e.close()
    n = 0
    for _key, (_hdr, d) in sorted(got.items()):
        for k in range(len(d["action"])):
            if n >= check:
                break
            a = int(d["action"][k])
            r = _two_ply_scores(weights_seed0, d["before"][k], int(d["mover"][k]), *d["dice"][k], k_top)
            if r[0] is None:   # fewer than 4 moves: 1-ply argmax
                v = r[1]
                assert v[a] >= v.max() - V_TOL
                continue
            cand, score, v = r
            if a not in set(cand.tolist()):
                # only a V tie at the top-4 boundary can move a candidate in or out
                assert abs(v[a] - v[cand[-1]]) < V_TOL, (a, v[a], v[cand[-1]])
                continue
            assert score[list(cand).index(a)] >= score.max() - 2 * V_TOL, (a, score)
            n += 1
    assert n >= check


def test_engine_2ply_kall_transitions(weights_seed0):
    from test_gpu_engine import _check_transitions, _collect
    e = _engine(weights_seed0, lanes=64, seed=13, ply=2, k_top=0)
    hdrs, recs = _collect(e, 150, chunk=75)
    e.close()
    assert _check_transitions(weights_seed0, hdrs, recs, 2) > 2000


def test_engine_2ply_k4_sampling_distribution(weights_seed0):
    """chi-square: the first decision of each lane (the opening position) is
    sampled from softmax(score / T) over the oracle's top-4 scores."""
    from bgx.episodes import decode_records
    e = _engine(weights_seed0, lanes=8192, seed=5, ply=2, k_top=4)
    e.step(1)
    e.step(299)
    h = e.harvest()
    e.close()
    d = decode_records(h.headers, h.records)
    init = golden("movegen_cases.npz")["boards"][0]
    groups = {}
    for k in np.nonzero(d["step"] == 0)[0]:
        if np.array_equal(d["before"][k], init):
            key = (int(d["mover"][k]), int(d["dice"][k][0]), int(d["dice"][k][1]))
            groups.setdefault(key, []).append(int(d["action"][k]))
    from scipy.stats import chisquare
    tested = 0
    for (mover, d0, d1), acts in sorted(groups.items(), key=lambda kv: -len(kv[1]))[:6]:
        cand, score, _v = _two_ply_scores(weights_seed0, init, mover, d0, d1, 4)
        p = np.exp((score - score.max()) / 1.5)
        p /= p.sum()
        pos = {int(c): j for j, c in enumerate(cand)}
        assert all(a in pos for a in acts)
        obs = np.bincount([pos[a] for a in acts], minlength=4)
        assert chisquare(obs, p * len(acts)).pvalue > 1e-4, (mover, d0, d1, obs, p)
        tested += 1
    assert tested >= 4
