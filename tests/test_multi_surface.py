"""The src/multi + src/environments surface kept for src/main.py (CPU only)."""
import multiprocessing
import queue

import numpy as np
import pytest
import torch

from environments import Episode, Experience, Player
from multi import ExperienceQueue, ParameterManager


@pytest.fixture(scope="module")
def manager():
    m = multiprocessing.Manager()
    yield m
    m.shutdown()


def test_parameter_manager_init_version_and_shapes(manager):
    pm = ParameterManager(manager.Lock(), manager.Value("i", 1), manager.dict())
    assert pm.get_version() == 1
    sd = pm.get_parameters()
    assert sd["fc1.weight"].shape == (128, 198) and sd["value_head.weight"].shape == (1, 128)
    assert sd["fc1.bias"].shape == (128,) and sd["value_head.bias"].shape == (1,)
    pm.set_parameters({k: v + 1 for k, v in sd.items()})
    assert pm.get_version() == 2
    np.testing.assert_allclose(pm.get_parameters()["fc1.bias"].numpy(), sd["fc1.bias"].numpy() + 1)


def test_temperature_schedule(manager):
    # parameter_manager.py:93-111: 1.5 at v<=1, linear to 0.5 at v >= 4001
    v = manager.Value("i", 1)
    pm = ParameterManager(manager.Lock(), v, manager.dict())
    assert pm.get_temperature() == 1.5
    v.value = 2001
    assert abs(pm.get_temperature() - 1.0) < 1e-12
    v.value = 4001
    assert pm.get_temperature() == 0.5
    v.value = 10 ** 6
    assert pm.get_temperature() == 0.5


def test_episode_counts_and_conversions():
    ep = Episode()
    obs = np.zeros(198, np.float32)
    for k, info in enumerate([{"current_player": Player.PLAYER1, "close_out_reward": True},
                              {"current_player": Player.PLAYER2},
                              {"current_player": Player.PLAYER1, "prime_reward": True},
                              {"current_player": Player.PLAYER2, "win_type": "gammon", "winner": Player.PLAYER2}]):
        ep.add_experience(Experience(obs, 0.1 * k, np.array(0.0, np.float32), k == 3, obs, 0.2), info)
    assert ep.win_type == "gammon"
    assert ep.close_out_counts == {Player.PLAYER1: 1, Player.PLAYER2: 0}
    assert ep.prime_reward_counts == {0: 1, 1: 0}   # IntEnum keys compare as ints
    ep.to_tensor(device="cpu")
    x = ep.experiences[3]
    assert x.observation.dtype == torch.float32 and x.state_value.dtype == torch.float32
    assert x.done.dtype == torch.int64   # the reference's int-before-bool dispatch (episode.py:39-42)


def test_experience_queue_roundtrip():
    q = ExperienceQueue()
    ep = Episode()
    q.put(ep)
    got = q.get(timeout=5)
    assert isinstance(got, Episode)
    with pytest.raises(queue.Empty):
        q.get(timeout=0.05)


def test_load_pth_round_trip(tmp_path):
    """A reference-format checkpoint (state_dict of BackgammonPolicyNetwork,
    parameter_manager.py:115-151) loads through bgx.ops.load_pth (weights_only)."""
    import torch
    from bgx.net import BackgammonPolicyNetwork
    from bgx.ops import load_pth
    torch.manual_seed(3)
    net = BackgammonPolicyNetwork()
    p = tmp_path / "ppo_backgammon.pth"
    torch.save(net.state_dict(), p)
    w = load_pth(str(p))
    sd = net.state_dict()
    np.testing.assert_array_equal(w["W1"], sd["fc1.weight"].numpy())
    np.testing.assert_array_equal(w["b1"], sd["fc1.bias"].numpy())
    np.testing.assert_array_equal(w["w2"], sd["value_head.weight"].numpy().reshape(128))
    np.testing.assert_array_equal(w["b2"], sd["value_head.bias"].numpy())


def test_seven_workers_cover_eight_gpus():
    """main.py:86 starts exactly 7 workers; gpus_for_worker spreads a node's
    GPUs over them (GPU g -> worker g mod 7: worker 0 drives GPUs 0 and 7),
    or follows BGX_GPU_MAP."""
    from multi.worker import gpus_for_worker
    got = [gpus_for_worker(i, 8) for i in range(7)]
    assert got == [[0, 7], [1], [2], [3], [4], [5], [6]]
    assert sorted(g for gs in got for g in gs) == list(range(8))
    assert [gpus_for_worker(i, 1) for i in range(7)] == [[0]] + [[]] * 6
    m = "0;1;2;3;4;5;6,7"
    assert [gpus_for_worker(i, 8, gpu_map=m) for i in range(7)] == [[0], [1], [2], [3], [4], [5], [6, 7]]
    assert gpus_for_worker(3, 8, gpu_map="0;1") == []
    import pytest
    with pytest.raises(ValueError):
        gpus_for_worker(0, 2, gpu_map="5")
