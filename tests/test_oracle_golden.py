"""Pin the CPU oracle (oracle/bgref.c) against the reference's golden vectors.

The fixtures were produced by tools/gen_golden.py importing the reference in
the build container; see that script's header for what was imported.
"""
import hashlib

import numpy as np
import pytest

from conftest import golden
import oracle as orc


def test_movegen_cases_ordered_with_submoves():
    d = golden("movegen_cases.npz")
    for i in range(len(d["boards"])):
        o0, o1 = d["offsets"][i], d["offsets"][i + 1]
        n, res, nsub, sub = orc.movegen(d["boards"][i], d["player"][i], *d["dice"][i],
                                        with_sub=True)
        assert n == o1 - o0, i
        np.testing.assert_array_equal(res, d["results"][o0:o1], err_msg=str(i))
        np.testing.assert_array_equal(nsub, d["nsub"][o0:o1])
        np.testing.assert_array_equal(sub, d["subs"][o0:o1])


def test_movegen_opening_counts():
    # P1 at the start: 3-1 -> 16, 6-6 -> 11, 1-1 -> 42, 6-5 -> 7, 2-1 -> 15
    init = golden("movegen_cases.npz")["boards"][0]
    for dice, cnt in (((3, 1), 16), ((6, 6), 11), ((1, 1), 42), ((6, 5), 7), ((2, 1), 15)):
        assert orc.movegen(init, 0, *dice)[0] == cnt


def test_movegen_digests():
    g = golden("movegen_digests.npz")
    for i in range(len(g["boards"])):
        n, res, _ = orc.movegen(g["boards"][i], g["player"][i], *g["dice"][i])
        assert n == g["count"][i], i
        assert hashlib.sha256(res.tobytes()).digest() == g["sha256"][i].tobytes(), i


def test_encode_live_and_interleaved_bit_exact():
    e = golden("encode.npz")
    live = orc.encode_many(e["boards"], e["player"], 0)
    np.testing.assert_array_equal(live.view(np.uint32), e["live"].view(np.uint32))
    n = len(e["interleaved"])
    inter = orc.encode_many(e["boards"][:n], e["player"][:n], 1)
    np.testing.assert_array_equal(inter.view(np.uint32), e["interleaved"].view(np.uint32))


@pytest.mark.parametrize("which", ["seed0", "ckpt"])
def test_value_within_1e5(which, weights_seed0, weights_ckpt):
    v = golden("value.npz")
    w = weights_seed0 if which == "seed0" else weights_ckpt
    ref = v["v_seed0"] if which == "seed0" else v["v_ckpt"]
    got = orc.value(w, v["x"])
    assert np.max(np.abs(got - ref)) < 1e-5


def test_reward_predicates():
    p = golden("predicates.npz")
    names = {"game_over": "check_game_over", "gammon": "check_for_gammon",
             "backgammon": "check_for_backgammon", "prime": "made_at_least_five_prime",
             "closed_out": "is_closed_out"}
    for key, fn in names.items():
        got = np.array([orc.predicate(fn, b, pl) for b, pl in zip(p["boards"], p["player"])])
        np.testing.assert_array_equal(got, p[key], err_msg=key)
    assert p["prime"].any() and p["closed_out"].any() and p["backgammon"].any()


def test_env_greedy_trajectories():
    t = golden("env_traj.npz")
    for (d0, dn, s0, sn) in t["episodes"]:
        env = orc.OracleEnv(t["dice"][d0:d0 + dn])
        env.reset()
        for s in range(s0, s0 + sn):
            np.testing.assert_array_equal(env.board, t["board"][s])
            assert env.env.current_player == t["player"][s]
            assert env.env.num_moves == t["num_moves"][s]
            assert env.env.full_moves == t["full_moves"][s]
            assert tuple(env.env.roll) == tuple(t["roll"][s])
            r = env.step(t["action"][s] if t["kind"][s] == 0 else 0)
            assert r.kind == t["kind"][s]
            assert np.float32(r.reward) == t["reward"][s]
            assert bool(r.done) == bool(t["done"][s])
            assert r.win_type == t["win_type"][s]
            assert bool(r.close_out_reward) == bool(t["close_out"][s])
            assert bool(r.prime_reward) == bool(t["prime"][s])
            if t["kind"][s] == 0:
                np.testing.assert_array_equal(env.board, t["after"][s])
                if not t["done"][s]:
                    mover = int(t["player"][s])
                    assert orc.predicate("is_closed_out", env.board, mover) == bool(t["closed_pred"][s])
                    assert orc.predicate("made_at_least_five_prime", env.board, mover) == bool(t["prime_pred"][s])


def _env_events(t):
    """Event counts of env_traj.npz (tools/gen_golden.py episode_events)."""
    k, rew = t["kind"], t["reward"]
    prev_pass = np.concatenate([[False], k[:-1] == 1])
    first = np.zeros(len(k), bool)
    first[t["episodes"][:, 2]] = True
    return dict(close_out=int(t["close_out"].sum()), prime=int(t["prime"].sum()),
                close_repeat=int((t["closed_pred"] & ~t["close_out"]).sum()),
                prime_repeat=int((t["prime_pred"] & ~t["prime"]).sum()),
                backgammon=int((t["win_type"] == 3).sum()), gammon=int((t["win_type"] == 2).sum()),
                pass_run=int(((k == 1) & prev_pass & ~first).sum()),
                shaping_rewards=sorted(set(rew[(rew > 0) & (rew < 1)].tolist())))


def test_env_fixture_covers_shaping_and_terminal_events():
    """The reference-generated trajectories hold every reward path of
    backgammon_env.py:167-213: close-outs (+0.30) and primes (+0.20), either
    predicate holding again after the player's reward was given (no second
    reward: once per player per game), gammons, backgammons, consecutive
    passes; under both weight sets (the seed-0 net and the 2.1M checkpoint)."""
    t = golden("env_traj.npz")
    ev = _env_events(t)
    assert ev["close_out"] >= 10 and ev["prime"] >= 10, ev
    assert ev["close_repeat"] >= 1 and ev["prime_repeat"] >= 1, ev
    assert ev["backgammon"] >= 3 and ev["gammon"] >= 3 and ev["pass_run"] >= 1, ev
    # the rewards are torch fp32 (backgammon_env.py:165-213): 0.2f and 0.3f exactly
    assert ev["shaping_rewards"] == [float(np.float32(0.2)), float(np.float32(0.3))], ev
    assert set(np.unique(t["weight_set"]).tolist()) == {0, 1}
    # the once-per-player rule: at most one close-out and one prime reward per player per game
    for (d0, dn, s0, sn) in t["episodes"]:
        rows = slice(s0, s0 + sn)
        for pl in (0, 1):
            mine = t["player"][rows] == pl
            assert t["close_out"][rows][mine].sum() <= 1 and t["prime"][rows][mine].sum() <= 1


def test_close_out_and_prime_never_coincide():
    """A step cannot earn both shaping rewards (0.30 + 0.20): a close-out needs
    the mover's six home points made (12 checkers), and a counted 5-prime needs
    an opponent checker past the prime's end (env_helper.py:167-242), i.e. on
    one of those home points, or 10 more checkers for a prime outside home.
    Checked exhaustively over the predicate fixture's boards and 20,000 random
    closed-out boards on the oracle."""
    p = golden("predicates.npz")
    assert not np.any(p["closed_out"] & p["prime"])
    rng = np.random.default_rng(5)
    n = 0
    for _ in range(20000):
        b = np.zeros(52, np.uint8)
        mover = int(rng.integers(2))
        home = np.arange(18, 24) if mover == 0 else np.arange(0, 6)
        b[24 * mover + home] = 2
        rest = 3
        while rest:
            i = int(rng.integers(24))
            if i in home or b[24 * (1 - mover) + i] == 0:
                k = int(rng.integers(1, rest + 1))
                b[24 * mover + i] += k
                rest -= k
        b[48 + (1 - mover)] = int(rng.integers(1, 4))
        left = 15 - b[48 + (1 - mover)]
        free = [i for i in range(24) if b[24 * mover + i] == 0]
        for i in rng.choice(free, size=min(len(free), 6), replace=False):
            k = int(min(left, rng.integers(1, 4)))
            b[24 * (1 - mover) + i] += k
            left -= k
        b[50 + (1 - mover)] = left
        if orc.predicate("is_closed_out", b, mover):
            n += 1
            assert not orc.predicate("made_at_least_five_prime", b, mover), b
    assert n == 20000


def test_two_ply_exact_mode(weights_seed0, weights_ckpt):
    t = golden("two_ply.npz")
    for i in range(len(t["boards"])):
        w0 = orc.two_ply_response(weights_seed0, t["boards"][i], t["opponent"][i])
        wc = orc.two_ply_response(weights_ckpt, t["boards"][i], t["opponent"][i])
        assert abs(w0 - t["w_seed0"][i]) < 1e-5
        assert abs(wc - t["w_ckpt"][i]) < 1e-5
