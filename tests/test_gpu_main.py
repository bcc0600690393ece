"""src/main.py's self-play plumbing on the GPU engine (tests/main_harness.py
restates main.py:65-91, 117-133): one worker process on cuda:0 behind the
reference's Manager / ParameterManager / ExperienceQueue surface delivers
Episodes whose Experiences are consistent with the oracle: V(s) and V(a)
within 1e-5 of the fp64 MLP on the decoded observations, next_observation's
indicator (the next player, the winner at a terminal step), the board chain
from one Experience to the next, terminal rewards, win types, and the field
types of Episode.to_tensor (episode.py:22-46: bool -> int64)."""
import os

import numpy as np
import pytest
import torch

import oracle as orc

pytestmark = pytest.mark.gpu
V_TOL = 1e-5


def _board_of(x):
    """Inverse of the live encoder (immutable_board.py:86-128): u8[52] + indicator."""
    x = np.asarray(x, np.float64)
    b = np.zeros(52, np.uint8)
    for pl in (0, 1):
        f = x[96 * pl:96 * pl + 96].reshape(24, 4)
        b[24 * pl:24 * pl + 24] = np.where(f[:, 3] > 0, 3 + 2 * f[:, 3], f[:, 0] + f[:, 1] + f[:, 2]).round()
    b[48], b[49] = round(x[192] * 2), round(x[194] * 2)
    b[50], b[51] = round(x[193] * 15), round(x[195] * 15)
    assert x[196] + x[197] == 1.0
    return b, int(x[197] == 1.0)


def test_main_loop_delivers_reference_episodes(weights_seed0, monkeypatch):
    from main_harness import run
    monkeypatch.setenv("BGX_LANES", "64")
    monkeypatch.setenv("BGX_STEPS_PER_HARVEST", "150")
    episodes, sd, _ = run(n_episodes=60)
    w = {"W1": sd["fc1.weight"].numpy(), "b1": sd["fc1.bias"].numpy(),
         "w2": sd["value_head.weight"].numpy().reshape(-1), "b2": sd["value_head.bias"].numpy()}
    n_exp = 0
    for ep in episodes:
        xs = ep.experiences
        assert len(xs) > 0
        for k, x in enumerate(xs):
            assert isinstance(x.observation, torch.Tensor) and x.observation.shape == (198,)
            assert x.observation.device.type == "cuda" and x.observation.dtype == torch.float32
            assert x.done.dtype == torch.int64          # episode.py:39-42, bool -> int64
            obs = x.observation.cpu().numpy()
            nxt = x.next_observation.cpu().numpy()
            b, p = _board_of(obs)
            a, q = _board_of(nxt)
            done = bool(x.done.item())
            assert q == (p if done else 1 - p)
            v = orc.value(w, np.stack([orc.encode(b, p), orc.encode(a, p)]))
            assert abs(v[0] - float(x.state_value)) < V_TOL
            assert abs(v[1] - float(x.next_state_value)) < V_TOL
            r = float(x.reward.item())
            if done:
                assert k == len(xs) - 1 and orc.predicate("check_game_over", a, p)
                assert r in (1.0, 2.0, 2.5)
            else:
                assert not orc.predicate("check_game_over", a, p) and r in (0.0, np.float32(0.2), np.float32(0.3),
                                                                            np.float32(0.5))
            if k + 1 < len(xs):   # passes move no checker
                nb, _ = _board_of(xs[k + 1].observation.cpu().numpy())
                np.testing.assert_array_equal(nb, a)
            n_exp += 1
        assert ep.win_type in (None, "regular", "gammon", "backgammon")
        assert (ep.win_type is None) == (not bool(xs[-1].done.item()))
    assert n_exp > 1000


class _PM:
    """ParameterManager stand-in (get_parameters / get_version / get_temperature)."""

    def __init__(self, w, version=1):
        self.w, self.v = w, version

    def get_parameters(self):
        return self.w

    def get_version(self):
        return self.v

    def get_temperature(self):
        return 1.5


def test_pipelined_worker_matches_engine(weights_seed0, monkeypatch):
    """multi/worker.py's pipelined cycle (each call queues the next launch and
    returns the previous launch's harvest) hands over exactly the engine's own
    harvests, one cycle late: call k's arrays equal a plain Engine's harvest
    after launch k - 1 (same seed, lanes and lane base as the worker's GPU 0),
    the first call returns none, and a version bump before a cycle steers that
    cycle's launch (the direct engine takes the new weights at the same point)."""
    from multi.worker import Worker
    from bgx import Engine
    monkeypatch.setenv("BGX_GPU_MAP", "0")
    monkeypatch.setenv("BGX_LANES", "96")
    monkeypatch.setenv("BGX_BALANCE", "0")        # lockstep launches: the harvests are run-independent
    monkeypatch.setenv("BGX_STEPS_PER_HARVEST", "60")
    w2 = {k: (v * 0.5 if k == "W1" else v) for k, v in weights_seed0.items()}
    pm = _PM(weights_seed0)
    wk = Worker(0, pm, None)
    got = []
    for k in range(5):
        if k == 3:
            pm.w, pm.v = w2, 2
        hdr, rec = wk.harvest_records()
        got.append((hdr.copy(), rec.copy()))
    torch.cuda.set_device(0)
    e = Engine(lanes=96, seed=1000003, lane_base=0, balance=False)
    e.set_weights(weights_seed0, temperature=1.5, version=1)
    want = []
    for k in range(4):
        if k == 3:
            e.set_weights(w2, temperature=1.5, version=2)
        e.step(60)
        h = e.harvest()
        want.append((h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32)))
    e.close()
    for e_ in wk.engines:
        e_.close()
    from bgx.records import episode_bounds

    def by_episode(hdr, rec):
        # headers come in the device's atomic append order (and word 2, the first
        # record, with it): compare per (lane, episode no.)
        offs, _ = episode_bounds(hdr)
        return {(int(r[0]), int(r[1])): (np.delete(r, 2), rec[offs[i]:offs[i + 1]]) for i, r in enumerate(hdr)}

    assert got[0][0].shape[0] == 0 and got[0][1].shape[0] == 0   # nothing finished before the first launch
    for k in range(4):
        a, b = by_episode(*got[k + 1]), by_episode(*want[k])
        assert a.keys() == b.keys(), f"episodes of launch {k}"
        for key in a:
            np.testing.assert_array_equal(a[key][0], b[key][0], err_msg=f"header {key} of launch {k}")
            np.testing.assert_array_equal(a[key][1], b[key][1], err_msg=f"records {key} of launch {k}")
    assert sum(g[0].shape[0] for g in got) > 20   # episodes finished (games end from ~50 steps)
