"""TD(0) trainer on device-resident episodes.

The reference's consumer (src/agents/trainer.py:10-166, Trainer.update) takes
exactly MIN_EPISODES_TO_TRAIN = 200 Episodes and, for each episode in turn:
Y = V(observations) (trainer.py:106-107), target = rewards with
gamma * Y[1:].detach() added to all but the last step (110-114), MSE loss
(117), zero_grad / backward (120-121), clip_grad_norm_(params, 1.0) (124-127),
the post-clip gradient norm as a metric (130-135), Adam step (lr 1e-3; the
configured LR decay is never applied in the reference) (138), then the new
state_dict goes to the ParameterManager (161).

DeviceTrainer.update_records() runs the same per-episode sequence straight
from the engine's compact records, and update(episodes) keeps the
reference's signature. backend="hip" (the default for records) runs the whole
update as one libbgx launch (bgx_td0_update, csrc/bgx_train.hip: weights in
registers, Adam moments in place, no host sync per episode); backend="torch"
runs it as eager torch ops (observations re-encoded with bgx_encode), the
checker the HIP path is tested against. batched=True (torch only) is a
flagged semantic change: one Adam step per update on the mean of the
per-episode losses.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import ops
from .records import WIN_TYPES
from .net import BackgammonPolicyNetwork

LEARNING_RATE = 1e-3          # config/configuration.py:17
GAMMA = 0.99                  # configuration.py:15
GRAD_CLIP_THRESHOLD = 1.0     # configuration.py:18
MIN_EPISODES_TO_TRAIN = 200   # configuration.py:7


class DeviceTrainer:
    def __init__(self, parameter_manager, device=None, lr=LEARNING_RATE, gamma=GAMMA,
                 grad_clip=GRAD_CLIP_THRESHOLD, batch_episode_size=MIN_EPISODES_TO_TRAIN, batched=False,
                 backend="hip"):
        self.parameter_manager = parameter_manager
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.policy_network = BackgammonPolicyNetwork().to(self.device)
        sd = {k: torch.as_tensor(v).to(self.device) for k, v in parameter_manager.get_parameters().items()}
        self.policy_network.load_state_dict(sd)
        self.optimizer = torch.optim.Adam(self.policy_network.parameters(), lr=lr)
        self.gamma = torch.tensor(gamma, device=self.device)
        self.grad_clip = grad_clip
        self.batch_episode_size = batch_episode_size
        self.batched = batched
        if backend not in ("hip", "torch"):
            raise ValueError(f"backend must be 'hip' or 'torch', not {backend!r}")
        self.backend = "torch" if batched else backend
        self.total_episodes = 0
        self._flat = None   # HIP backend state: params / Adam m / v (flat, state_dict order), step

    # ------------------------------------------------------------ inputs
    def _from_records(self, headers, records):
        """(observations [m, 198], rewards [m], episode lengths, win types) on the device."""
        rec = torch.as_tensor(records).to(self.device)
        if rec.dtype != torch.int32:
            rec = rec.view(torch.int32) if rec.dtype == torch.uint32 else rec.to(torch.int32)
        before = torch.zeros((rec.shape[0], 8), dtype=torch.int32, device=self.device)
        before[:, :7] = rec[:, :7]   # the board before the move, the mover's indicator (bgx/records.py)
        obs = ops.encode_packed(before)
        rewards = rec[:, 9].contiguous().view(torch.float32)
        hdr = np.asarray(torch.as_tensor(headers).cpu().numpy()).astype(np.uint32)
        lens = hdr[:, 3].astype(np.int64).tolist()
        wins = [WIN_TYPES[int(w) & 0xFF] for w in (hdr[:, 5] & 0xFF).tolist()]
        return obs, rewards, lens, wins

    def _from_episodes(self, episodes):
        obs, rew, lens, wins = [], [], [], []
        for ep in episodes:
            obs.extend(torch.as_tensor(np.asarray(x.observation, np.float32)) for x in ep.experiences)
            rew.extend(float(np.asarray(x.reward)) for x in ep.experiences)
            lens.append(len(ep.experiences))
            wins.append(ep.win_type)
        obs_t = torch.stack(obs).to(self.device) if obs else torch.zeros((0, 198), device=self.device)
        return obs_t, torch.tensor(rew, dtype=torch.float32, device=self.device), lens, wins

    # ------------------------------------------------------------ update
    def update(self, episodes):
        """Trainer.update(episodes) (trainer.py:49-166): exactly batch_episode_size episodes."""
        if len(episodes) != self.batch_episode_size:
            raise ValueError(f"Expected {self.batch_episode_size} episodes, but got {len(episodes)}.")
        return self._update(*self._from_episodes(episodes))

    def update_records(self, headers, records):
        """The same update from compact records (headers [n, 16], records [m, 12],
        each episode's records contiguous in header order); any n >= 1."""
        if self.backend == "hip":
            return self._update_hip(headers, records)
        return self._update(*self._from_records(headers, records))

    # ------------------------------------------------------------ HIP backend
    _KEYS = ("fc1.weight", "fc1.bias", "value_head.weight", "value_head.bias")

    def _hip_state(self):
        """Flat fp32 params / Adam moments (state_dict order) and the step count,
        taken over from the torch module / optimizer the first time."""
        if self._flat is not None and self._flat.get("token") != self._module_token():
            self._flat = None   # the module / optimizer changed outside the HIP updates: take it over again
        if self._flat is None:
            net, opt = self.policy_network, self.optimizer
            params = [dict(net.named_parameters())[k] for k in self._KEYS]
            flat = torch.cat([p.detach().reshape(-1) for p in params]).contiguous()
            m = torch.zeros_like(flat)
            v = torch.zeros_like(flat)
            step = 0
            st = [opt.state.get(p, {}) for p in params]
            if all("exp_avg" in x for x in st):
                m = torch.cat([x["exp_avg"].reshape(-1) for x in st]).contiguous()
                v = torch.cat([x["exp_avg_sq"].reshape(-1) for x in st]).contiguous()
                step = int(float(st[0]["step"]))
            self._flat = {"p": flat, "m": m, "v": v,
                          "step": torch.tensor([step], dtype=torch.int32, device=self.device),
                          "token": self._module_token()}
        return self._flat

    def _module_token(self):
        """Identifies the module's parameters and the optimizer's moments as the
        HIP backend last left them: every in-place write (load_state_dict,
        copy_, an optimizer step) bumps a tensor's _version, and replacing the
        optimizer state swaps the moment tensors."""
        net, opt = self.policy_network, self.optimizer
        params = [dict(net.named_parameters())[k] for k in self._KEYS]
        st = [opt.state.get(p, {}) for p in params]
        return (tuple(p._version for p in params),
                tuple((id(x.get("exp_avg")), id(x.get("exp_avg_sq")), id(x.get("step"))) for x in st))

    def _sync_module(self):
        """Copy the HIP backend's weights / moments back into the torch module and
        optimizer (state_dict consumers, and a later torch-backend update)."""
        f = self._flat
        net, opt = self.policy_network, self.optimizer
        params = [dict(net.named_parameters())[k] for k in self._KEYS]
        o = 0
        step = int(f["step"].item())
        with torch.no_grad():
            for p in params:
                n = p.numel()
                p.copy_(f["p"][o:o + n].view_as(p))
                if step > 0:
                    st = opt.state[p]
                    st["exp_avg"] = f["m"][o:o + n].view_as(p).clone()
                    st["exp_avg_sq"] = f["v"][o:o + n].view_as(p).clone()
                    st["step"] = torch.tensor(float(step))
                o += n
        f["token"] = self._module_token()

    def _update_hip(self, headers, records):
        from ._lib import check, lib, ptr, stream_handle
        rec = torch.as_tensor(records).to(self.device)
        if rec.dtype != torch.int32:
            rec = rec.view(torch.int32) if rec.dtype == torch.uint32 else rec.to(torch.int32)
        rec = rec.contiguous()
        hdr = np.asarray(torch.as_tensor(headers).cpu().numpy()).astype(np.uint32)
        lens = hdr[:, 3].astype(np.int64)
        if len(lens) and int(lens.max()) > 2048:
            raise ValueError("bgx_td0_update: an episode has more than 2048 records")
        if len(lens) and int(lens.min()) <= 0:
            # the kernel skips an empty episode (no Adam step), while the metrics
            # below divide by every episode: reject it instead of skewing them
            raise ValueError("bgx_td0_update: an episode has no records")
        offs = torch.as_tensor(np.concatenate([[0], np.cumsum(lens)]).astype(np.int32), device=self.device)
        f = self._hip_state()
        metrics = torch.zeros(5, dtype=torch.float64, device=self.device)
        n_eps = len(lens)
        clip = float(self.grad_clip) if self.grad_clip is not None else 0.0
        with torch.cuda.device(self.device):   # the trainer's device and its current stream
            check(lib().bgx_td0_update(ptr(rec), ptr(offs), n_eps, ptr(f["p"]), ptr(f["m"]), ptr(f["v"]),
                                       ptr(f["step"]), float(self.optimizer.param_groups[0]["lr"]),
                                       float(self.gamma), clip, ptr(metrics),
                                       stream_handle(torch.cuda.current_stream(self.device))),
                  "bgx_td0_update")
        self.total_episodes += n_eps
        self._sync_module()
        a = metrics.tolist()
        win_counts = {"regular": 0, "gammon": 0, "backgammon": 0}
        for w in (hdr[:, 5] & 0xFF).tolist():
            name = WIN_TYPES[int(w)]
            if name in win_counts:
                win_counts[name] += 1
        self.parameter_manager.set_parameters(self.policy_network.state_dict())
        out = {"loss": a[0], "grad_norm": a[1], "td_error": a[2], "predicted_value": a[3], "reward": a[4],
               "episode_length": float(lens.sum())}
        out = {k: v / max(1, n_eps) for k, v in out.items()}
        out["win_counts"] = win_counts
        out["episodes"] = n_eps
        return out

    def _update(self, obs, rewards, lens, wins):
        if self._flat is not None:   # continue from the HIP backend's state
            self._sync_module()
            self._flat = None
        net, opt = self.policy_network, self.optimizer
        params = list(net.parameters())
        n_eps = len(lens)
        self.total_episodes += n_eps
        m = {"loss": 0.0, "td_error": 0.0, "grad_norm": 0.0, "predicted_value": 0.0, "reward": 0.0,
             "episode_length": 0.0}
        win_counts = {"regular": 0, "gammon": 0, "backgammon": 0}
        offs = np.concatenate([[0], np.cumsum(lens)]).tolist()
        # metrics accumulate on the device; one host read per update
        acc = torch.zeros(6, dtype=torch.float64, device=self.device)
        if self.batched:
            losses = []
            for e in range(n_eps):
                y, tgt = self._episode_terms(obs, rewards, offs[e], offs[e + 1])
                losses.append(F.mse_loss(y, tgt))
            opt.zero_grad()
            loss = torch.stack(losses).mean()
            loss.backward()
            if self.grad_clip is not None:
                torch.nn.utils.clip_grad_norm_(params, self.grad_clip)
            opt.step()
            acc[0] = loss.detach() * n_eps
        else:
            for e in range(n_eps):
                y, tgt = self._episode_terms(obs, rewards, offs[e], offs[e + 1])
                loss = F.mse_loss(y, tgt)
                opt.zero_grad()
                loss.backward()
                if self.grad_clip is not None:
                    pre = torch.nn.utils.clip_grad_norm_(params, self.grad_clip)
                    # the reference measures the norm after clipping (trainer.py:130-135):
                    # torch scales by min(1, clip / (norm + 1e-6))
                    post = pre * torch.clamp(self.grad_clip / (pre + 1e-6), max=1.0)
                else:
                    post = torch.norm(torch.stack([p.grad.detach().norm(2) for p in params if p.grad is not None]), 2)
                opt.step()
                yd = y.detach()
                acc += torch.stack([loss.detach().double(), post.double(), (tgt - yd).abs().mean().double(),
                                    yd.mean().double(), rewards[offs[e]:offs[e + 1]].sum().double(),
                                    torch.zeros((), dtype=torch.float64, device=self.device)])
        a = acc.tolist()
        m["loss"], m["grad_norm"], m["td_error"], m["predicted_value"], m["reward"] = a[0], a[1], a[2], a[3], a[4]
        m["episode_length"] = float(offs[-1])
        for w in wins:
            if w in win_counts:
                win_counts[w] += 1
        self.parameter_manager.set_parameters(net.state_dict())
        out = {k: v / max(1, n_eps) for k, v in m.items()}
        out["win_counts"] = win_counts
        out["episodes"] = n_eps
        return out

    def _episode_terms(self, obs, rewards, a, b):
        y = self.policy_network(obs[a:b]).squeeze()
        tgt = rewards[a:b].clone().squeeze()
        if b - a > 1:
            tgt[:-1] += self.gamma * y[1:].detach()
        return y, tgt
