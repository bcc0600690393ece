"""Device TD(0) trainer vs a line-by-line fp32 CPU
restatement of the reference's Trainer.update loop (src/agents/trainer.py:81-138;
the reference module itself needs pynvml / boto3 / tensorboardX, absent here)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden

pytestmark = pytest.mark.gpu


class _PM:
    def __init__(self, sd):
        self.sd = {k: v.clone() for k, v in sd.items()}
        self.version = 1

    def get_parameters(self, device=None):
        return {k: v.to(device) if device else v for k, v in self.sd.items()}

    def set_parameters(self, sd):
        self.sd = {k: v.detach().cpu().clone() for k, v in sd.items()}
        self.version += 1


def _reference_update(sd, episodes, lr=1e-3, gamma=0.99, clip=1.0):
    """trainer.py:81-138 restated (CPU, fp32): per episode forward, TD(0)
    target, MSE, backward, clip_grad_norm_, Adam step."""
    from bgx.net import BackgammonPolicyNetwork
    net = BackgammonPolicyNetwork()
    net.load_state_dict(sd)
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    g = torch.tensor(gamma)
    for ep in episodes:
        obs = torch.stack([torch.as_tensor(x.observation) for x in ep.experiences])
        rew = torch.stack([torch.as_tensor(x.reward) for x in ep.experiences]).squeeze()
        y = net(obs).squeeze()
        tgt = rew.clone()
        if len(ep.experiences) > 1:
            tgt[:-1] += g * y[1:].detach()
        loss = F.mse_loss(y, tgt)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), clip)
        opt.step()
    return net.state_dict()


def test_device_trainer_matches_reference_loop(weights_seed0):
    from bgx import Engine
    from bgx.episodes import to_episodes
    from bgx.net import BackgammonPolicyNetwork
    from bgx.trainer import DeviceTrainer
    from environments import Episode, Experience, Player
    eng = Engine(lanes=512, seed=9)
    eng.set_weights(weights_seed0, 1.5, 1)
    eng.step(300)
    h = eng.harvest()
    eng.close()
    eps = to_episodes(h, Episode, Experience, Player)[:40]
    n_rec = sum(len(e.experiences) for e in eps)
    hdr = h.headers[:40].cpu()
    rec = h.records[:n_rec]
    torch.manual_seed(0)
    sd0 = BackgammonPolicyNetwork().state_dict()

    pm_a, pm_b = _PM(sd0), _PM(sd0)
    ta = DeviceTrainer(pm_a, device="cuda", batch_episode_size=len(eps), backend="torch")
    tb = DeviceTrainer(pm_b, device="cuda", batch_episode_size=len(eps), backend="torch")
    ma = ta.update_records(hdr, rec)
    tb.update(eps)
    for k in sd0:   # records path == Episode-object path, bit for bit
        torch.testing.assert_close(pm_a.sd[k], pm_b.sd[k], rtol=0, atol=0)
    ref = _reference_update(sd0, eps)
    for k in sd0:   # GPU vs CPU fp32 over 40 sequential Adam steps
        torch.testing.assert_close(pm_a.sd[k], ref[k], rtol=1e-4, atol=2e-5)
    assert ma["episodes"] == len(eps) and pm_a.version == 2
    assert ma["episode_length"] == pytest.approx(n_rec / len(eps))
    with pytest.raises(ValueError):
        tb.update(eps[:3])   # trainer.py:49-52: exactly batch_episode_size episodes


def test_hip_trainer_matches_torch_and_reference(weights_seed0):
    """bgx_td0_update (one launch over the episodes, csrc/bgx_train.hip) against
    the torch backend and the CPU fp32 restatement of trainer.py:81-138: the
    same weights after 2 x 40 sequential per-episode Adam steps (summation
    orders differ: tolerance), the same metrics, and the Adam state carried
    from one update to the next (and into a torch-backend update)."""
    from bgx import Engine
    from bgx.episodes import to_episodes
    from bgx.net import BackgammonPolicyNetwork
    from bgx.trainer import DeviceTrainer
    from environments import Episode, Experience, Player
    eng = Engine(lanes=512, seed=11)
    eng.set_weights(weights_seed0, 1.5, 1)
    eng.step(300)
    h = eng.harvest()
    eng.close()
    eps = to_episodes(h, Episode, Experience, Player)[:80]
    lens = [len(e.experiences) for e in eps]
    hdr = h.headers[:80].cpu()
    rec = h.records[:sum(lens)]
    torch.manual_seed(1)
    sd0 = BackgammonPolicyNetwork().state_dict()
    pm_h, pm_t = _PM(sd0), _PM(sd0)
    th = DeviceTrainer(pm_h, device="cuda", batch_episode_size=40, backend="hip")
    tt = DeviceTrainer(pm_t, device="cuda", batch_episode_size=40, backend="torch")
    n0 = sum(lens[:40])
    mh = th.update_records(hdr[:40], rec[:n0])
    mt = tt.update_records(hdr[:40], rec[:n0])
    for k in sd0:
        torch.testing.assert_close(pm_h.sd[k], pm_t.sd[k], rtol=1e-4, atol=2e-5)
    for k in ("loss", "grad_norm", "td_error", "predicted_value", "reward", "episode_length"):
        assert mh[k] == pytest.approx(mt[k], rel=1e-4, abs=1e-6), k
    assert mh["win_counts"] == mt["win_counts"] and mh["episodes"] == 40
    # second update: the Adam moments / step continue on the device
    th.update_records(hdr[40:80], rec[n0:])
    tt.update_records(hdr[40:80], rec[n0:])
    for k in sd0:
        torch.testing.assert_close(pm_h.sd[k], pm_t.sd[k], rtol=2e-4, atol=4e-5)
    ref = _reference_update(sd0, eps)
    for k in sd0:   # 80 sequential Adam steps, GPU (one launch per 40) vs CPU fp32
        torch.testing.assert_close(pm_h.sd[k], ref[k], rtol=2e-4, atol=4e-5)
    # the module / optimizer state follow the device state: a torch-backend
    # update continues from it
    th.backend = "torch"
    th.update_records(hdr[:40], rec[:n0])
    tt.update_records(hdr[:40], rec[:n0])
    for k in sd0:
        torch.testing.assert_close(pm_h.sd[k], pm_t.sd[k], rtol=3e-4, atol=6e-5)


def test_hip_trainer_takes_outside_module_changes(weights_seed0):
    """A load_state_dict on the module between two HIP updates is not
    overwritten by the backend's flat copy (the next update starts from the
    loaded weights, as the torch backend does), and an episode with no
    records is rejected instead of skewing the metrics."""
    from bgx import Engine
    from bgx.net import BackgammonPolicyNetwork
    from bgx.trainer import DeviceTrainer
    eng = Engine(lanes=512, seed=13)
    eng.set_weights(weights_seed0, 1.5, 1)
    eng.step(300)
    h = eng.harvest()
    eng.close()
    hdr = h.headers[:20].cpu()
    n = int(hdr[:, 3].sum())
    rec = h.records[:n]
    torch.manual_seed(2)
    sd0 = BackgammonPolicyNetwork().state_dict()
    torch.manual_seed(3)
    sd1 = BackgammonPolicyNetwork().state_dict()
    pm_h, pm_t = _PM(sd0), _PM(sd1)
    th = DeviceTrainer(pm_h, device="cuda", batch_episode_size=20, backend="hip")
    tt = DeviceTrainer(pm_t, device="cuda", batch_episode_size=20, backend="hip")
    th.update_records(hdr, rec)
    th.policy_network.load_state_dict(sd1)          # an outside write (e.g. a checkpoint restore)
    th.optimizer.state.clear()
    th.update_records(hdr, rec)
    tt.update_records(hdr, rec)                     # a fresh trainer from sd1
    for k in sd0:
        torch.testing.assert_close(pm_h.sd[k], pm_t.sd[k], rtol=0, atol=0)
    bad = hdr.clone()
    bad[0, 3] = 0
    with pytest.raises(ValueError, match="no records"):
        th.update_records(bad, rec)
