"""GPU engine parity: every harvested Experience is replayed through the CPU oracle.

The engine's dice and sampling streams cannot match the reference's
(np.random / torch.distributions), so the check is per transition: the
recorded (board, mover, dice) must generate — in the oracle, which is pinned
to the reference — the recorded afterstate at the recorded action index, and
V(s), V(a), reward, done, win type and shaping flags must equal what the
oracle computes for that transition (worker.py:101-162, backgammon_env.py:130-221).
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


def _collect(e, steps, chunk=100):
    from bgx.episodes import decode_records
    hdrs, recs = [], []
    done = 0
    while done < steps:
        k = min(chunk, steps - done)
        e.step(k)
        h = e.harvest()
        hdr = h.headers.cpu().numpy().view(np.uint32)
        hdrs.append(hdr)
        recs.append(decode_records(hdr, h.records))
        done += k
    e.sync()
    return hdrs, recs


def _check_transitions(weights, hdrs, recs, ply):
    """Every record against the oracle: afterstate, V(s) / V(a), reward, done,
    win type, shaping; the 198-d observation (mover's indicator) and
    next_observation (the next player's, or the winner's at a terminal step,
    backgammon_env.py:196-218), bit for bit; who moves after pass turns."""
    n_checked = 0
    for hdr, d in zip(hdrs, recs):
        o = 0
        for row in hdr:
            n = int(row[3])
            flags = 0
            for k in range(o, o + n):
                b, mover, dice = d["before"][k], int(d["mover"][k]), d["dice"][k]
                cnt, res, _ = orc.movegen(b, mover, int(dice[0]), int(dice[1]))
                assert d["n_moves"][k] == min(cnt, 4095) and cnt > 0
                a = int(d["action"][k])
                assert 0 <= a < min(cnt, 500)
                np.testing.assert_array_equal(res[a], d["after"][k])
                xs = orc.encode_many(np.stack([b, res[a]]), [mover, mover])
                v = orc.value(weights, xs)
                assert abs(v[0] - d["v_s"][k]) < V_TOL and abs(v[1] - d["v_a"][k]) < V_TOL
                np.testing.assert_array_equal(d["obs"][k], xs[0])
                nxt = mover if d["done"][k] else 1 - mover
                np.testing.assert_array_equal(d["next_obs"][k], orc.encode(res[a], nxt))
                if k + 1 < o + n:   # the other player moves next, each pass turn flips again
                    passes = int(d["step"][k + 1]) - int(d["step"][k]) - 1
                    assert passes >= 0
                    assert int(d["mover"][k + 1]) == (1 - mover) ^ (passes & 1), (k, passes)
                # reward / terminal / shaping (env_helper.py:113-242, backgammon_env.py:167-213)
                after = res[a]
                if orc.predicate("check_game_over", after, mover):
                    wt = 3 if orc.predicate("check_for_backgammon", after, mover) else (
                        2 if orc.predicate("check_for_gammon", after, mover) else 1)
                    assert d["done"][k] and d["win_type"][k] == wt
                    assert d["reward"][k] == np.float32({1: 1.0, 2: 2.0, 3: 2.5}[wt])
                    assert k == o + n - 1
                else:
                    assert not d["done"][k]
                    r = np.float32(0.0)
                    co = orc.predicate("is_closed_out", after, mover) and not (flags >> mover) & 1
                    pr = orc.predicate("made_at_least_five_prime", after, mover) and not (flags >> (2 + mover)) & 1
                    if co:
                        r = np.float32(r + np.float32(0.30))
                        flags |= 1 << mover
                    if pr:
                        r = np.float32(r + np.float32(0.20))
                        flags |= 4 << mover
                    assert bool(d["close_out"][k]) == bool(co) and bool(d["prime"][k]) == bool(pr)
                    assert d["reward"][k] == r
                if k > o:   # passes never change the board
                    np.testing.assert_array_equal(d["before"][k], d["after"][k - 1])
                n_checked += 1
            if n:
                assert d["step"][o] >= 0
                last = o + n - 1
                if d["done"][last]:   # the terminal step ends the episode: steps = its step + 1
                    assert int(row[4]) == int(d["step"][last]) + 1
                    assert int(row[5]) & 0xFF == int(d["win_type"][last])
                    assert (int(row[5]) >> 8) & 0xFF == int(d["mover"][last])
            assert int(row[4]) <= 300
            assert int(row[4]) == 300 or (n > 0 and d["done"][o + n - 1])
            o += n
    return n_checked


def test_engine_1ply_transitions_match_oracle(weights_seed0):
    e = _engine(weights_seed0, lanes=512, seed=11, ply=1)
    hdrs, recs = _collect(e, 400)
    assert sum(len(h) for h in hdrs) > 100
    assert _check_transitions(weights_seed0, hdrs, recs, 1) > 10000
    st = e.stats()
    assert st["env_steps"] == 512 * 400
    e.close()


def test_engine_episode_starts_from_reset(weights_seed0):
    e = _engine(weights_seed0, lanes=256, seed=5, ply=1)
    hdrs, recs = _collect(e, 300)
    init = golden("movegen_cases.npz")["boards"][0]
    for hdr, d in zip(hdrs, recs):
        o = 0
        for row in hdr:
            n = int(row[3])
            if n and int(row[1]) > 0:   # every episode after the lane's first starts at the reset
                np.testing.assert_array_equal(d["before"][o], init)
                assert d["dice"][o][0] != d["dice"][o][1]   # first roll re-rolled off doubles
            o += n
    e.close()


def test_engine_sampling_distribution(weights_seed0):
    """chi-square: the first decision of each lane is sampled from softmax(V/T)."""
    from bgx.episodes import decode_records
    e = _engine(weights_seed0, lanes=16384, seed=3, ply=1)
    e.step(1)
    e.sync()
    # the first step of every lane is a decision from the initial board
    e.step(299)
    h = e.harvest()
    d = decode_records(h.headers, h.records)
    first = d["step"] == 0
    init = golden("movegen_cases.npz")["boards"][0]
    groups = {}
    for k in np.nonzero(first)[0]:
        if not np.array_equal(d["before"][k], init):
            continue
        key = (int(d["mover"][k]), int(d["dice"][k][0]), int(d["dice"][k][1]))
        groups.setdefault(key, []).append(int(d["action"][k]))
    from scipy.stats import chisquare
    tested = 0
    for (mover, d0, d1), acts in groups.items():
        if len(acts) < 200:
            continue
        cnt, res, _ = orc.movegen(init, mover, d0, d1)
        v = orc.value(weights_seed0, orc.encode_many(res, [mover] * cnt))
        p = np.exp((v - v.max()) / 1.5)
        p /= p.sum()
        obs = np.bincount(acts, minlength=cnt)
        assert chisquare(obs, p * len(acts)).pvalue > 1e-4, (mover, d0, d1)
        tested += 1
    assert tested >= 3
    e.close()


def test_engine_2ply_k4_transitions(weights_seed0):
    e = _engine(weights_seed0, lanes=128, seed=21, ply=2, k_top=4)
    hdrs, recs = _collect(e, 200)
    assert _check_transitions(weights_seed0, hdrs, recs, 2) > 1000
    # chosen action is one of the top-4 by 1-ply V whenever >= 4 moves exist
    for hdr, d in zip(hdrs, recs):
        for k in range(len(d["action"])):
            cnt = int(d["n_moves"][k])
            if cnt < 4:
                continue
            _, res, _ = orc.movegen(d["before"][k], int(d["mover"][k]), *d["dice"][k])
            res = res[:500]
            v = orc.value(weights_seed0, orc.encode_many(res, [int(d["mover"][k])] * len(res)))
            top4 = np.argsort(-v, kind="stable")[:4]
            assert int(d["action"][k]) in set(top4.tolist())
    e.close()


def test_two_ply_exact_mode_vs_reference(weights_seed0, weights_ckpt):
    from bgx import ops
    t = golden("two_ply.npz")
    for w, key in ((weights_seed0, "w_seed0"), (weights_ckpt, "w_ckpt")):
        net = ops.Net(w)
        W = net.two_ply(torch.from_numpy(t["boards"]).cuda(), torch.from_numpy(t["opponent"]).cuda())
        np.testing.assert_allclose(W.cpu().numpy(), t[key], atol=V_TOL, rtol=0)


ROLLS21 = [(a, b) for a in range(1, 7) for b in range(a, 7)]   # DICE_ROLLS order (two_ply.py:10-32)
P21 = np.array([1.0 if a == b else 2.0 for a, b in ROLLS21]) / 36.0
SMALL_DOUBLES = (0, 6, 11)                                      # 1-1, 2-2, 3-3 (two_ply.py:119-121)


def _reply_values(weights, board, opp, r):
    a, b = ROLLS21[r]
    n, res, _ = orc.movegen(board, opp, a, b)
    return orc.value(weights, orc.encode_many(res, [opp] * n)) if n else np.zeros(0)


def test_two_ply_reference_sampled_mode(weights_seed0):
    """two_ply.py:119-121 (random.sample of 50 replies for 1-1 / 2-2 / 3-3) as
    bgx_two_ply_sampled: reproducible per seed; equal to the exact mode where
    no such roll has more than 50 replies; never above it (a subset's top-5
    mean is at most the full set's); its mean over seeds matches the mean over
    numpy random 50-subsets of the oracle's reply values."""
    from bgx import ops
    t = golden("two_ply.npz")
    net = ops.Net(weights_seed0)
    B, O = torch.from_numpy(t["boards"]).cuda(), torch.from_numpy(t["opponent"]).cuda()
    exact = net.two_ply(B, O).cpu().numpy()
    s = net.two_ply(B, O, sample=50, seed=3).cpu().numpy()
    np.testing.assert_array_equal(s, net.two_ply(B, O, sample=50, seed=3).cpu().numpy())
    assert np.all(s <= exact + 1e-12)
    affected = []
    for i in range(len(exact)):
        big = [r for r in SMALL_DOUBLES
               if len(_reply_values(weights_seed0, t["boards"][i], int(t["opponent"][i]), r)) > 50]
        if big:
            affected.append((i, big))
        else:
            assert s[i] == exact[i], i
    assert affected, "the fixture holds positions with > 50 replies to a small double"
    rng = np.random.default_rng(0)
    for i, big in affected[:2]:
        seeds = 200
        draws = net.two_ply(B[i:i + 1].repeat(seeds, 1), O[i:i + 1].repeat(seeds), sample=50, seed=11).cpu().numpy()
        assert len(np.unique(draws)) > 1   # jobs of the batch draw different subsets
        mu, var = exact[i], 0.0
        for r in big:
            v = _reply_values(weights_seed0, t["boards"][i], int(t["opponent"][i]), r)
            full = np.sort(v)[::-1][:5].mean()
            sub = np.array([np.sort(rng.choice(v, 50, replace=False))[::-1][:5].mean() for _ in range(3000)])
            mu += P21[r] * (sub.mean() - full)
            var += P21[r] ** 2 * sub.var()
        assert abs(draws.mean() - mu) < 5 * np.sqrt(var / seeds) + 1e-6, (i, draws.mean(), mu, np.sqrt(var / seeds))


def test_engine_2ply_reference_sampled_mode(weights_seed0):
    """Engine(reply_sample=50): the reference-sampled 2-ply keeps every
    transition valid and the chosen action among the top-4 by 1-ply V."""
    e = _engine(weights_seed0, lanes=64, seed=4, ply=2, k_top=4, reply_sample=50)
    hdrs, recs = _collect(e, 60, chunk=30)
    e.close()
    assert _check_transitions(weights_seed0, hdrs, recs, 2) > 200


def _by_episode(hdrs, recs):
    """{(lane, episode no.): (header words 2.., {field: records})} — header
    order is the device's atomic append order, so runs compare per episode."""
    out = {}
    for hdr, d in zip(hdrs, recs):
        o = 0
        for row in hdr:
            n = int(row[3])
            out[(int(row[0]), int(row[1]))] = (row[3:].copy(), {k: v[o:o + n] for k, v in d.items()})
            o += n
    return out


@pytest.mark.parametrize("ply", [1, 2])
def test_graph_launch_matches_direct_launch(ply, monkeypatch):
    """The graph-captured step sequence (BGX_GRAPH=1) and direct launches
    (the default) produce identical episodes and records for the same seed."""
    w = {k: golden("weights_seed0.npz")[k] for k in ("W1", "b1", "w2", "b2")}
    runs = []
    for g in ("1", "0"):
        monkeypatch.setenv("BGX_GRAPH", g)
        e = _engine(w, lanes=256, seed=11, ply=ply, k_top=4, fused=False)
        runs.append(_by_episode(*_collect(e, 120 if ply == 1 else 40, chunk=40)))
        e.close()
    a, b = runs
    assert len(a) > 0 and a.keys() == b.keys()
    for key in a:
        np.testing.assert_array_equal(a[key][0], b[key][0], err_msg=str(key))
        for f in a[key][1]:
            np.testing.assert_array_equal(a[key][1][f], b[key][1][f], err_msg=f"{key} {f}")


def test_bulk_queue_episodes_equal_direct_path(weights_seed0):
    """put_records -> shared-memory ring -> get() decodes (on the GPU) the same
    Episodes as the worker-side to_episodes path."""
    from bgx.episodes import to_episodes
    from environments import Episode, Experience, Player
    from multi.experience_queue import ExperienceQueue
    e = _engine(weights_seed0, lanes=256, seed=3, ply=1)
    e.step(150)
    h = e.harvest()
    direct = to_episodes(h, Episode, Experience, Player)
    assert len(direct) > 10
    q = ExperienceQueue(capacity_mb=64)
    try:
        assert q.put_records(h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32))
        assert q.qsize() == len(direct)
        bulk = [q.get(timeout=10) for _ in range(len(direct))]
        assert q.qsize() == 0
    finally:
        q.close()
        e.close()
    for a, b in zip(direct, bulk):
        assert a.win_type == b.win_type
        assert a.close_out_counts == b.close_out_counts and a.prime_reward_counts == b.prime_reward_counts
        assert len(a.experiences) == len(b.experiences)
        for x, y in zip(a.experiences, b.experiences):
            np.testing.assert_array_equal(x.observation, y.observation)
            np.testing.assert_array_equal(x.next_observation, y.next_observation)
            assert x.state_value == y.state_value and x.next_state_value == y.next_state_value
            assert x.reward == y.reward and x.done == y.done


def test_engine_greedy_picks_the_highest_value(weights_ckpt):
    """greedy=True (play_versus_ai.py:188-195): the chosen afterstate has the
    largest V among the legal candidates (within the V tolerance), checked
    against the oracle's fp64 values on the shipped checkpoint."""
    e = _engine(weights_ckpt, lanes=128, seed=21, ply=1, greedy=True)
    hdrs, recs = _collect(e, 150, chunk=50)
    e.close()
    n = 0
    for d in recs:
        for k in range(len(d["action"])):
            b, mover, dice = d["before"][k], int(d["mover"][k]), d["dice"][k]
            cnt, res, _ = orc.movegen(b, mover, int(dice[0]), int(dice[1]))
            m = min(cnt, 500)
            v = orc.value(weights_ckpt, orc.encode_many(res[:m], [mover] * m))
            a = int(d["action"][k])
            assert v[a] >= v.max() - V_TOL, (k, a, v[a], v.max())
            n += 1
    assert n > 2000


def _same_runs(a, b):
    assert len(a) > 0 and a.keys() == b.keys()
    for key in a:
        np.testing.assert_array_equal(a[key][0], b[key][0], err_msg=str(key))
        for f in a[key][1]:
            np.testing.assert_array_equal(a[key][1][f], b[key][1][f], err_msg=f"{key} {f}")


@pytest.mark.parametrize("tier,fl", [("", "16"), ("", "32"), ("2", "16"), ("3", "32")])
def test_fused_step_matches_phased_engine(weights_seed0, tier, fl, monkeypatch):
    """The fused 1-ply kernel (one persistent launch per step() call, 16 or 32
    lanes per workgroup: BGX_FUSED_LANES) and the phased engine (movegen / MLP /
    select launches per step) produce identical episodes and records for the
    same seed: same afterstates in the same order, V with the same bits, same
    samples. With BGX_MG_TEST_TIER=2/3 every fused movegen job is redone by the
    workgroup tiers (32 KB slice, or the global workspace)."""
    lanes, steps = (300, 160) if not tier else (48, 60)
    ref = _engine(weights_seed0, lanes=lanes, seed=17, ply=1, fused=False)
    a = _by_episode(*_collect(ref, steps, chunk=40))
    ref.close()
    monkeypatch.setenv("BGX_FUSED_LANES", fl)
    if tier:
        monkeypatch.setenv("BGX_MG_TEST_TIER", tier)
    e = _engine(weights_seed0, lanes=lanes, seed=17, ply=1, fused=True)
    assert e.fused
    b = _by_episode(*_collect(e, steps, chunk=40))
    st = e.stats()
    e.close()
    _same_runs(a, b)
    assert st["env_steps"] == lanes * steps
    if tier:
        assert st["fallback_jobs"] > 0


def test_2ply_tier1_kernels_agree(weights_seed0, monkeypatch):
    """2-ply K=4 (128 lanes: 10,752 reply jobs per step) with the reply launch
    on the 16-wave block kernel (BGX_MG_FEW=1) and on the balanced pool
    kernel (the default for large launches): identical episodes and records
    (the reply rows land at different flat offsets; V, the top-5 means and
    the picks do not change)."""
    runs = []
    for few in ("1", "0"):
        monkeypatch.setenv("BGX_MG_FEW", few)
        e = _engine(weights_seed0, lanes=128, seed=5, ply=2, k_top=4)
        runs.append(_by_episode(*_collect(e, 60, chunk=30)))
        e.close()
    _same_runs(runs[0], runs[1])


@pytest.mark.parametrize("fl", ["16", "32"])
def test_fused_greedy_and_ragged_lanes(weights_ckpt, fl, monkeypatch):
    """A lane count that is not a multiple of 16 / 32 (the last workgroup is
    partly empty) and greedy play: fused == phased on the shipped checkpoint."""
    runs = []
    monkeypatch.setenv("BGX_FUSED_LANES", fl)
    for fused in (False, True):
        e = _engine(weights_ckpt, lanes=37, seed=9, ply=1, greedy=True, fused=fused)
        runs.append(_by_episode(*_collect(e, 200, chunk=50)))
        e.close()
    _same_runs(*runs)


@pytest.mark.parametrize("fl", ["16", "32"])
def test_fused_balanced_launch_keeps_every_lane_game(weights_seed0, fl, monkeypatch):
    """balance=True (include/bgx.h bgx_config.balance): step(n) runs n x lanes
    lane-steps in total with the workgroups at their own pace. Every lane's
    games are unchanged — each (lane, episode) both runs finished has identical
    records — and the launch's lane-step total is the budget plus less than
    one workgroup-step per workgroup."""
    monkeypatch.setenv("BGX_FUSED_LANES", fl)
    lanes, steps, chunk = 300, 200, 40
    ref = _engine(weights_seed0, lanes=lanes, seed=23, ply=1, fused=True)
    a = _by_episode(*_collect(ref, steps, chunk=chunk))
    ref.close()
    e = _engine(weights_seed0, lanes=lanes, seed=23, ply=1, fused=True, balance=True)
    b = _by_episode(*_collect(e, steps, chunk=chunk))
    st = e.stats()
    e.close()
    groups = (lanes + int(fl) - 1) // int(fl)
    launches = steps // chunk
    assert lanes * steps <= st["env_steps"] < lanes * steps + launches * groups * int(fl)
    common = a.keys() & b.keys()
    assert len(common) >= 0.8 * min(len(a), len(b)) and len(common) > 100
    for key in common:
        np.testing.assert_array_equal(a[key][0], b[key][0], err_msg=str(key))
        for f in a[key][1]:
            np.testing.assert_array_equal(a[key][1][f], b[key][1][f], err_msg=f"{key} {f}")


def test_fused_in_kernel_harvest_slots(weights_seed0):
    """The fused engine harvests inside its launches (each workgroup appends
    its own lanes' finished episodes at the end of a launch, bgx_fused.hip):
    two launches between tickets accumulate into one harvest, a ticket with no
    launch since the previous one is empty, and a ticket's arrays stay intact
    until the second harvest_enqueue after it although the launches after the
    next ticket already harvest (three slots). The episodes equal the phased
    engine's (which harvests with its own kernels) record for record."""
    from bgx.episodes import decode_records
    ref = _engine(weights_seed0, lanes=96, seed=31, ply=1, fused=False)
    want = _by_episode(*_collect(ref, 200, chunk=40))
    ref.close()
    e = _engine(weights_seed0, lanes=96, seed=31, ply=1, fused=True)
    hdrs, recs = [], []

    def take(t):
        h = e.harvest_fetch(t)
        hdr = h.headers.cpu().numpy().view(np.uint32)
        hdrs.append(hdr)
        recs.append(decode_records(hdr, h.records))
        return hdr.shape[0]

    e.step(40)
    e.step(40)                  # two launches, one harvest
    t0 = e.harvest_enqueue()
    t1 = e.harvest_enqueue()    # nothing ran since t0
    e.step(40)                  # harvests into t2's slot while t0 / t1 are unread
    assert take(t0) > 0
    assert take(t1) == 0
    t2 = e.harvest_enqueue()
    e.step(40)                  # t3's slot
    t3 = e.harvest_enqueue()
    e.step(40)                  # t4's slot = t1's: t2 and t3 must still be intact
    assert take(t2) > 0 and take(t3) > 0
    take(e.harvest_enqueue())
    e.close()
    got = _by_episode(hdrs, recs)
    assert len(got) > 50 and got.keys() == want.keys()
    for key in want:
        np.testing.assert_array_equal(got[key][0], want[key][0], err_msg=str(key))
        for f in want[key][1]:
            np.testing.assert_array_equal(got[key][1][f], want[key][1][f], err_msg=f"{key} {f}")


def test_fused_harvest_past_capacity_is_an_error(weights_seed0):
    """Several fused launches without a harvest finish more episodes than a
    small output holds (ep_cap = 64 headers): a workgroup whose episodes do
    not fit copies nothing and keeps them in its lanes' rings for the next
    ticket; once the rings overflow (ring = 512) the episodes are lost and the
    fetch reports BGX_E_CAPACITY (flag 8). Only the overflowing lanes are
    dropped; the engine keeps running and harvests normally afterwards."""
    from bgx import BgxError
    e = _engine(weights_seed0, lanes=64, seed=5, ply=1, fused=True, ep_cap=64, ring=512)
    for _ in range(5):
        e.step(200)
    with pytest.raises(BgxError, match=r"\(-3\).*flags 0x8"):
        e.harvest()
    e.step(40)
    h = e.harvest()
    assert 0 < h.n_episodes <= 64
    e.sync()
    e.close()


def test_fused_over_capacity_episodes_wait_for_the_next_ticket(weights_seed0):
    """A launch whose finished episodes exceed the ticket's output (ep_cap)
    keeps the groups that do not fit in the rings; the next ticket delivers
    them. Over both tickets every (lane, episode) equals an engine with room
    for all, and nothing is reported lost."""
    ref = _engine(weights_seed0, lanes=128, seed=8, ply=1, fused=True)
    ref.step(200)
    h = ref.harvest()
    from bgx.episodes import decode_records
    hdr = h.headers.cpu().numpy().view(np.uint32)
    want = _by_episode([hdr], [decode_records(hdr, h.records)])
    ref.close()
    e = _engine(weights_seed0, lanes=128, seed=8, ply=1, fused=True, ep_cap=150)
    e.step(200)                 # ~280 episodes finish; the output holds 150 headers
    hs, rs = [], []
    for _ in range(3):          # the held groups come with the following (empty-launch) tickets
        h = e.harvest()
        hdr = h.headers.cpu().numpy().view(np.uint32)
        assert hdr.shape[0] <= 150
        hs.append(hdr)
        rs.append(decode_records(hdr, h.records))
        e.step(1)
    e.sync()
    e.close()
    got = _by_episode(hs, rs)
    assert len(want) > 150
    assert want.keys() <= got.keys()
    for key in want:
        np.testing.assert_array_equal(got[key][0], want[key][0], err_msg=str(key))
        for f in want[key][1]:
            np.testing.assert_array_equal(got[key][1][f], want[key][1][f], err_msg=f"{key} {f}")


@pytest.mark.parametrize("fused", [True, False])
def test_fetch_reports_only_its_tickets_flags(weights_seed0, fused):
    """Error flags belong to the ticket whose launches raised them:
    with the next launch already queued behind a failing ticket, fetching the
    failing ticket reports its flags, and the next ticket (whose launch was in
    flight during that fetch) reports none."""
    from bgx import BgxError
    # no harvest: the 512-slot rings overflow (flag 8); the fused engine harvests
    # inside every launch, so its output is made small (ep_cap) to keep episodes
    # in the rings (test_fused_harvest_past_capacity_is_an_error)
    e = _engine(weights_seed0, lanes=64, seed=5, ply=1, fused=fused, ring=512, **({"ep_cap": 64} if fused else {}))
    for _ in range(4):
        e.step(200)
    t0 = e.harvest_enqueue()
    e.step(40)                  # in flight while t0 is fetched
    t1 = e.harvest_enqueue()
    with pytest.raises(BgxError, match="flags 0x8"):
        e.harvest_fetch(t0)
    if fused:
        # the small output cannot drain the rings, so lanes may overflow again
        # during t1's own launch: t1 reports only such flags of its own
        try:
            e.harvest_fetch(t1)
        except BgxError as ex:
            assert "flags 0x8" in str(ex)
        e.close()
        return
    h = e.harvest_fetch(t1)
    assert h.n_episodes >= 0
    e.step(40)
    e.harvest()
    e.sync()
    e.close()


@pytest.mark.parametrize("fused", [True, False])
def test_pipelined_harvest_equals_synchronous(weights_seed0, fused):
    """harvest_enqueue / harvest_fetch (the next step queued before the host
    reads a harvest; three rotating buffers) deliver exactly the episodes of
    the synchronous harvest(); a stale ticket is refused."""
    from bgx import BgxError
    a = _engine(weights_seed0, lanes=96, seed=29, ply=1, fused=fused)
    want = _by_episode(*_collect(a, 200, chunk=40))
    a.close()
    from bgx.episodes import decode_records
    b = _engine(weights_seed0, lanes=96, seed=29, ply=1, fused=fused)
    hdrs, recs, pend = [], [], None
    for _ in range(5):
        b.step(40)
        t = b.harvest_enqueue()
        if pend is not None:
            h = b.harvest_fetch(pend)
            hdr = h.headers.cpu().numpy().view(np.uint32)
            hdrs.append(hdr)
            recs.append(decode_records(hdr, h.records))
        pend = t
    h = b.harvest_fetch(pend)
    hdr = h.headers.cpu().numpy().view(np.uint32)
    hdrs.append(hdr)
    recs.append(decode_records(hdr, h.records))
    with pytest.raises(BgxError, match="ticket"):
        b.harvest_fetch(pend - 2)
    b.close()
    _same_runs(want, _by_episode(hdrs, recs))
