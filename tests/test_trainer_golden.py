"""Trainer parity pinned by the reference (tests/golden/trainer.npz, made by
tools/gen_golden.py --only trainer: the reference's own Trainer.update,
src/agents/trainer.py:48-166, on 200 synthetic episodes stored as the
engine's compact records, with no-op stand-ins for its telemetry imports).

CPU: the fp32 restatement of the update loop that the GPU trainer tests use
as their checker (tests/test_gpu_trainer.py::_reference_update), fed the
records decoded on the host and encoded by the oracle, gives the reference's
weights. GPU: DeviceTrainer (HIP backend: one bgx_td0_update launch; torch
backend) on the same records gives the reference's weights and metrics."""
import numpy as np
import pytest
import torch

from conftest import golden

KEYS = ("fc1.weight", "fc1.bias", "value_head.weight", "value_head.bias")


def _sd(prefix):
    g = golden("trainer.npz")
    return {k: torch.from_numpy(g[prefix + k.replace(".", "_")].copy()) for k in KEYS}


def _episodes():
    """(observations per episode [n, 198] float32, rewards per episode) from the
    fixture's records: the before-board and the mover (bgx/records.py), encoded
    by the oracle (immutable_board.py:86-128)."""
    import oracle as orc
    g = golden("trainer.npz")
    hdr, rec = g["headers"], g["records"]
    w = rec[:, :7].astype(np.uint32)
    b = np.zeros((len(rec), 52), np.uint8)
    for k in range(6):
        for q in range(8):
            b[:, 8 * k + q] = (w[:, k] >> (4 * q)) & 15
    for i in range(4):
        b[:, 48 + i] = (w[:, 6] >> (4 * i)) & 15
    mover = ((w[:, 6] >> 16) & 1).astype(np.uint8)
    x = orc.encode_many(b, mover).astype(np.float32)
    r = rec[:, 9].copy().view(np.float32)
    out, o = [], 0
    for n in hdr[:, 3].astype(int):
        out.append((torch.from_numpy(x[o:o + n]), torch.from_numpy(r[o:o + n])))
        o += n
    return out


def test_restated_update_equals_reference_fixture():
    """The restated loop (per episode: forward, TD(0) target with gamma V[t+1]
    detached, MSE, backward, clip_grad_norm_(1.0), Adam lr 1e-3) reproduces
    the reference's weights after 200 sequential updates on the CPU."""
    import torch.nn.functional as F
    from bgx.net import BackgammonPolicyNetwork
    torch.set_num_threads(1)
    net = BackgammonPolicyNetwork()
    net.load_state_dict(_sd("init_"))
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    g = torch.tensor(0.99)
    for obs, rew in _episodes():
        y = net(obs).squeeze()
        tgt = rew.clone().squeeze()
        if obs.shape[0] > 1:
            tgt[:-1] += g * y[1:].detach()
        loss = F.mse_loss(y, tgt)
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 1.0)
        opt.step()
    want = _sd("after_")
    sd = net.state_dict()
    for k in KEYS:
        torch.testing.assert_close(sd[k], want[k], rtol=1e-5, atol=1e-6)


class _PM:
    def __init__(self, sd):
        self.sd = {k: v.clone() for k, v in sd.items()}

    def get_parameters(self, device=None):
        return {k: v.to(device) if device else v for k, v in self.sd.items()}

    def set_parameters(self, sd):
        self.sd = {k: v.detach().cpu().clone() for k, v in sd.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("backend", ["hip", "torch"])
def test_device_trainer_equals_reference_fixture(backend):
    """DeviceTrainer.update_records on the fixture's 200 episodes (8,942
    records): the reference's state_dict after its update, within the
    tolerance of 200 sequential fp32 Adam steps summed in another order, and
    its logged metrics (trainer.py:156-163, 187-217)."""
    from bgx.trainer import DeviceTrainer
    g = golden("trainer.npz")
    pm = _PM(_sd("init_"))
    t = DeviceTrainer(pm, device="cuda", batch_episode_size=200, backend=backend)
    m = t.update_records(torch.from_numpy(g["headers"].astype(np.int64)),
                         torch.from_numpy(g["records"].view(np.int32)))
    want = _sd("after_")
    for k in KEYS:
        torch.testing.assert_close(pm.sd[k], want[k], rtol=5e-4, atol=1e-4)
    for k in ("loss", "td_error", "grad_norm", "predicted_value", "reward", "episode_length"):
        assert m[k] == pytest.approx(float(g["metric_" + k]), rel=2e-4, abs=1e-6), k
    wc = g["win_counts"]
    assert m["win_counts"] == {"regular": int(wc[0]), "gammon": int(wc[1]), "backgammon": int(wc[2])}
    assert m["episodes"] == 200
