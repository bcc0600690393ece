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


def test_two_ply_exact_mode(weights_seed0, weights_ckpt):
    t = golden("two_ply.npz")
    for i in range(len(t["boards"])):
        w0 = orc.two_ply_response(weights_seed0, t["boards"][i], t["opponent"][i])
        wc = orc.two_ply_response(weights_ckpt, t["boards"][i], t["opponent"][i])
        assert abs(w0 - t["w_seed0"][i]) < 1e-5
        assert abs(wc - t["w_ckpt"][i]) < 1e-5
