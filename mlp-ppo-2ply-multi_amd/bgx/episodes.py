"""Harvested compact records -> the reference's Episode / Experience objects.

Experience fields after Episode.to_numpy() (src/environments/episode.py:5-46,
src/multi/worker.py:149-168): observation / next_observation np.float32[198]
(features of the board with the indicator of the player to move, or of the
winner at a terminal step), state_value / next_state_value Python floats,
reward np.float32 0-d array, done bool. Episode carries win_type and
close_out_counts / prime_reward_counts keyed by the players who made a
decision (episode.py:56-76). Observations are re-encoded on the GPU from the
packed boards (bgx_encode_packed), not stored as 198 floats per step.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops
from . import records as records_np
from .engine import Harvest
from .records import REC_WORDS, WIN_TYPES


def decode_records(headers, records: torch.Tensor):
    """Harvested episodes -> dict of host numpy arrays: the record fields
    (bgx/records.py) plus the boards before / after every move (u8 [m, 52])
    and the 198-d observations, encoded on the device (bgx_encode_packed).
    headers: uint32/int32 [n, 16] (host or device); records int32 [m, 12]
    (device), each episode's records contiguous in header order."""
    hdr = headers.cpu().numpy() if isinstance(headers, torch.Tensor) else np.asarray(headers)
    m = records.shape[0]
    if m == 0:
        z = np.zeros((0, 198), np.float32)
        out = {k: v for k, v in records_np.fields(np.zeros((0, REC_WORDS), np.uint32)).items()}
        out.update(obs=z, next_obs=z, before=np.zeros((0, 52), np.uint8), after=np.zeros((0, 52), np.uint8))
        return out
    rec = records.cpu().numpy()
    before, after = records_np.packed_before_after(hdr, rec)
    dev = records.device
    b_t = torch.from_numpy(before.view(np.int32)).to(dev)
    a_t = torch.from_numpy(after.view(np.int32)).to(dev)
    out = records_np.fields(rec)
    # engine-produced boards: the unchecked, asynchronous packed encoder
    out.update(obs=ops.encode_packed(b_t).cpu().numpy(), next_obs=ops.encode_packed(a_t).cpu().numpy(),
               before=ops.unpack(b_t).cpu().numpy(), after=ops.unpack(a_t).cpu().numpy())
    return out


def to_episodes(h: Harvest, episode_cls, experience_cls, player_enum):
    """Build reference-shaped Episode objects (already in to_numpy() form)."""
    return episodes_from_arrays(h.headers.cpu().numpy().astype(np.uint32), h.records, episode_cls,
                                experience_cls, player_enum)


def episodes_from_arrays(hdr, records, episode_cls, experience_cls, player_enum):
    """hdr uint32 [n, 16] (host), records int32 [m, 12] (device) -> Episodes.
    Field types follow Episode.to_numpy() (episode.py:22-46): observation
    np.float32[198] views, state values Python floats, reward a 0-d np.float32
    array, done bool."""
    d = decode_records(hdr, records)
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
