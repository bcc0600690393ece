"""Harvested compact records -> the reference's Episode / Experience objects.

Experience fields after Episode.to_numpy() (src/environments/episode.py:5-46,
src/multi/worker.py:149-168): observation / next_observation np.float32[198]
(features of the board with the indicator of the player to move, or of the
winner at a terminal step), state_value / next_state_value Python floats,
reward np.float32 0-d array, done bool. Episode carries win_type and
close_out_counts / prime_reward_counts keyed by the players who made a
decision (episode.py:56-76). Observations are re-encoded on the GPU from the
packed boards (bgx_encode), not stored as 198 floats per step.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from .engine import WIN_TYPES, Harvest


def decode_records(records: torch.Tensor):
    """records int32 [m, 24] (device) -> dict of host numpy arrays, with the
    198-d observations encoded on the device."""
    m = records.shape[0]
    if m == 0:
        z = np.zeros((0, 198), np.float32)
        return dict(obs=z, next_obs=z, v_s=np.zeros(0, np.float32), v_a=np.zeros(0, np.float32),
                    reward=np.zeros(0, np.float32), done=np.zeros(0, bool), action=np.zeros(0, np.int32),
                    n_moves=np.zeros(0, np.int32), dice=np.zeros((0, 2), np.int32),
                    close_out=np.zeros(0, bool), prime=np.zeros(0, bool), mover=np.zeros(0, np.int32),
                    win_type=np.zeros(0, np.int32), before=np.zeros((0, 52), np.uint8),
                    after=np.zeros((0, 52), np.uint8), step=np.zeros(0, np.int32))
    before, after = records[:, 0:8].contiguous(), records[:, 8:16].contiguous()
    b8, a8 = ops.unpack(before), ops.unpack(after)
    obs = ops.encode(b8, ops.packed_player(before))
    nxt = ops.encode(a8, ops.packed_player(after))
    tail = records[:, 16:24].cpu().numpy()
    f = tail[:, 0:3].copy().view(np.float32)
    w3, w4 = tail[:, 3].astype(np.uint32), tail[:, 4].astype(np.uint32)
    return dict(
        obs=obs.cpu().numpy(), next_obs=nxt.cpu().numpy(), v_s=f[:, 0], v_a=f[:, 1], reward=f[:, 2],
        action=(w3 & 0xFFFF).astype(np.int32), n_moves=(w3 >> 16).astype(np.int32),
        dice=np.stack([(w4 & 0xFF), (w4 >> 8) & 0xFF], 1).astype(np.int32),
        done=((w4 >> 16) & 1).astype(bool), close_out=((w4 >> 17) & 1).astype(bool),
        prime=((w4 >> 18) & 1).astype(bool), mover=((w4 >> 19) & 1).astype(np.int32),
        win_type=((w4 >> 20) & 7).astype(np.int32), before=b8.cpu().numpy(), after=a8.cpu().numpy(),
        step=tail[:, 6].astype(np.int32))


def to_episodes(h: Harvest, episode_cls, experience_cls, player_enum):
    """Build reference-shaped Episode objects (already in to_numpy() form)."""
    return episodes_from_arrays(h.headers.cpu().numpy().astype(np.uint32), h.records, episode_cls,
                                experience_cls, player_enum)


def episodes_from_arrays(hdr, records, episode_cls, experience_cls, player_enum):
    """hdr uint32 [n, 8] (host), records int32 [m, 24] (device) -> Episodes.
    Field types follow Episode.to_numpy() (episode.py:22-46): observation
    np.float32[198] views, state values Python floats, reward a 0-d np.float32
    array, done bool."""
    d = decode_records(records)
    obs, nxt = d["obs"], d["next_obs"]
    v_s, v_a, done = d["v_s"].tolist(), d["v_a"].tolist(), d["done"].tolist()
    rew = d["reward"].astype(np.float32).reshape(-1, 1)
    mover, win, close, prime = d["mover"].tolist(), d["win_type"].tolist(), d["close_out"].tolist(), d["prime"].tolist()
    players = [player_enum(0), player_enum(1)]
    eps = []
    o = 0
    for row in hdr.tolist():
        n = int(row[3])
        ep = episode_cls()
        for k in range(o, o + n):
            ex = experience_cls(observation=obs[k], state_value=v_s[k], reward=rew[k].reshape(()),
                                done=done[k], next_observation=nxt[k], next_state_value=v_a[k])
            pl = players[mover[k]]
            info = {"current_player": pl}
            if win[k]:
                info["win_type"] = WIN_TYPES[win[k]]
                info["winner"] = pl
            if close[k]:
                info["close_out_reward"] = True
            if prime[k]:
                info["prime_reward"] = True
            ep.add_experience(ex, info)
        o += n
        eps.append(ep)
    return eps
