"""The engine's harvest wire format (include/bgx.h, bgx_harvest) as numpy.

Experience record, REC_WORDS = 12 uint32 (48 B):
  0..6  the board before the move, packed (word 6 bit 16 = the mover)
  7     V(s) f32          8  V(a) f32          9  reward f32
  10    action | n_moves << 11 | step << 23
  11    dice0 | dice1 << 3 | done << 6 | close_out << 7 | prime << 8 |
        mover << 9 | win_type << 10
Episode header, EP_WORDS = 16 uint32 (64 B):
  global lane, episode no., first record, n_records, env steps,
  win_type | winner << 8 | flags << 16, final board words 0..6, 0, 0, 0
The board after record k's move (Experience.next_observation) is record
k + 1's before-board (passes move no checker), and for an episode's last
record the header's final board; its indicator is the mover at a terminal
step (the winner) and the other player otherwise (backgammon_env.py:196-218).
Pure numpy so the CPU side (queue, gather, tests) needs no GPU.
"""
from __future__ import annotations

import numpy as np

REC_WORDS = 12
EP_WORDS = 16
WIN_TYPES = {0: None, 1: "regular", 2: "gammon", 3: "backgammon"}


def fields(rec: np.ndarray) -> dict:
    """Scalar fields of records uint32/int32 [m, 12] (host)."""
    r = np.ascontiguousarray(rec).view(np.uint32).reshape(-1, REC_WORDS)
    f = r[:, 7:10].copy().view(np.float32)
    w10, w11 = r[:, 10], r[:, 11]
    return dict(
        v_s=f[:, 0], v_a=f[:, 1], reward=f[:, 2],
        action=(w10 & 0x7FF).astype(np.int32), n_moves=((w10 >> 11) & 0xFFF).astype(np.int32),
        step=(w10 >> 23).astype(np.int32),
        dice=np.stack([w11 & 7, (w11 >> 3) & 7], 1).astype(np.int32),
        done=((w11 >> 6) & 1).astype(bool), close_out=((w11 >> 7) & 1).astype(bool),
        prime=((w11 >> 8) & 1).astype(bool), mover=((w11 >> 9) & 1).astype(np.int32),
        win_type=((w11 >> 10) & 3).astype(np.int32))


def episode_bounds(headers: np.ndarray):
    """(offsets [n + 1], lengths [n]) of the episodes' contiguous records."""
    h = np.ascontiguousarray(headers).view(np.uint32).reshape(-1, EP_WORDS)
    lens = h[:, 3].astype(np.int64)
    return np.concatenate([[0], np.cumsum(lens)]), lens


def packed_before_after(headers: np.ndarray, rec: np.ndarray):
    """Packed boards [m, 8] before and after every record's move (host numpy),
    with the indicator of Experience.observation / next_observation."""
    r = np.ascontiguousarray(rec).view(np.uint32).reshape(-1, REC_WORDS)
    h = np.ascontiguousarray(headers).view(np.uint32).reshape(-1, EP_WORDS)
    m = r.shape[0]
    offs, lens = episode_bounds(h)
    if offs[-1] != m:
        raise ValueError(f"headers count {offs[-1]} records, got {m}")
    before = np.zeros((m, 8), np.uint32)
    before[:, :7] = r[:, :7]
    after = np.zeros((m, 8), np.uint32)
    after[:-1] = before[1:]
    has = lens > 0
    after[offs[1:][has] - 1, :7] = h[has, 6:13]
    f = fields(r)
    flag = np.where(f["done"], f["mover"], 1 - f["mover"]).astype(np.uint32)
    after[:, 6] = (after[:, 6] & 0xFFFF) | (flag << 16)
    return before, after


def pack_record(before_w, mover, v_s, v_a, reward, action, n_moves, step, dice, done, close_out, prime,
                win_type):
    """One record (uint32 [12]) from its fields (tests, synthetic inputs)."""
    r = np.zeros(REC_WORDS, np.uint32)
    r[:7] = np.asarray(before_w, np.uint32)[:7]
    r[6] = (r[6] & 0xFFFF) | (np.uint32(mover) << 16)
    r[7:10] = np.array([v_s, v_a, reward], np.float32).view(np.uint32)
    r[10] = (int(action) & 0x7FF) | (min(int(n_moves), 4095) << 11) | (min(int(step), 511) << 23)
    r[11] = (int(dice[0]) | (int(dice[1]) << 3) | (int(done) << 6) | (int(close_out) << 7) | (int(prime) << 8)
             | (int(mover) << 9) | (int(win_type) << 10))
    return r
