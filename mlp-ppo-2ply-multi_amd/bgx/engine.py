"""The self-play engine: thousands of game lanes on one MI355X.

Replaces, per device, the reference's pool of CPU workers (src/main.py:86-91,
src/multi/worker.py:17-179): every lane is one BackgammonEnv
(src/environments/backgammon_env.py) driven by the worker's episode loop.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import torch

from ._lib import Config, HarvestInfo, Stats, check, lib, require_cuda, stream_handle
from .ops import weights_from
from .records import EP_WORDS, REC_WORDS, WIN_TYPES  # noqa: F401  (wire format, include/bgx.h)


@dataclass
class Harvest:
    """Finished episodes: headers int32 [n, 16] and records int32 [m, 12] on the
    engine's device (layouts in include/bgx.h, bgx_harvest; bgx/records.py)."""
    headers: torch.Tensor
    records: torch.Tensor

    @property
    def n_episodes(self):
        return int(self.headers.shape[0])

    @property
    def n_records(self):
        return int(self.records.shape[0])


class Engine:
    def __init__(self, lanes=4096, seed=0, ply=1, k_top=4, device=None, lane_base=0, alpha=1.0,
                 beta=0.9, max_steps=300, max_legal=500, ring=1024, ep_cap=0, cand_per_lane=256,
                 reply_per_lane=0, greedy=False, fused=True, reply_sample=0, balance=False):
        require_cuda()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        cfg = Config()
        lib().bgx_config_default(ctypes.byref(cfg))
        cfg.lanes, cfg.lane_base, cfg.seed = int(lanes), int(lane_base), int(seed)
        cfg.ply, cfg.k_top, cfg.alpha, cfg.beta = int(ply), int(k_top), float(alpha), float(beta)
        cfg.max_steps, cfg.max_legal, cfg.ring, cfg.ep_cap = int(max_steps), int(max_legal), int(ring), int(ep_cap)
        cfg.cand_per_lane, cfg.reply_per_lane = int(cand_per_lane), int(reply_per_lane)
        cfg.greedy = 1 if greedy else 0
        cfg.fused = 1 if fused else 0   # 1-ply: one persistent launch per step() call
        cfg.reply_sample = int(reply_sample)   # 2-ply: 0 exact, 50 = two_ply.py:119-121 random.sample
        cfg.balance = 1 if balance else 0   # fused 1-ply: step(n) = n x lanes lane-steps (include/bgx.h)
        self.cfg = cfg
        self.lanes = int(lanes)
        self.fused = bool(fused) and int(ply) == 1
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().bgx_engine_create(self.device.index, ctypes.byref(cfg), ctypes.byref(h)),
                  "bgx_engine_create")
        self._h = h
        self._empty = None
        self.version = 0
        self.temperature = None

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib().bgx_engine_destroy(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def max_steps_per_call(self):
        return self.cfg.ring - self.cfg.max_steps

    def set_weights(self, weights, temperature=1.5, version=1):
        W1, b1, w2, b2 = weights_from(weights)
        fp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        check(lib().bgx_set_weights(self._h, fp(W1), fp(b1), fp(w2), fp(b2), float(temperature),
                                    int(version)), "bgx_set_weights")
        self.version, self.temperature = int(version), float(temperature)

    def set_dice(self, dice):
        """Test hook (bgx_engine_set_dice): scripted single-die draws, uint8
        [lanes, k] in 1..6, two per roll, replacing np.random.randint(1, 7)
        (backgammon_env.py:310-311); needs greedy=True. Every lane restarts
        from the reset with its own draws."""
        import numpy as np
        d = np.ascontiguousarray(np.asarray(dice, dtype=np.uint8).reshape(self.lanes, -1))
        check(lib().bgx_engine_set_dice(self._h, d.ctypes.data_as(ctypes.c_void_p), int(d.shape[1])),
              "bgx_engine_set_dice")

    def step(self, n=1, stream=None):
        """Advance every lane by n env steps (asynchronous on the stream);
        balance=True: n x lanes lane-steps in total, faster lanes run ahead."""
        check(lib().bgx_step(self._h, int(n), stream_handle(stream)), "bgx_step")

    def sync(self):
        check(lib().bgx_sync(self._h), "bgx_sync")

    def harvest(self, stream=None, clone=True) -> Harvest:
        info = HarvestInfo()
        check(lib().bgx_harvest(self._h, ctypes.byref(info), stream_handle(stream)), "bgx_harvest")
        return self._harvest_from(info, clone)

    def harvest_enqueue(self, stream=None) -> int:
        """Queue a harvest behind the last step and return its ticket at once
        (bgx_harvest_enqueue): the next step() can be launched before the host
        looks at the result."""
        t = ctypes.c_int(0)
        check(lib().bgx_harvest_enqueue(self._h, ctypes.byref(t), stream_handle(stream)), "bgx_harvest_enqueue")
        return int(t.value)

    def harvest_fetch(self, ticket: int, clone=False, wrap=True):
        """Wait for a queued harvest (one of the last two tickets). Without
        clone the tensors alias the engine's buffers, valid until the second
        harvest_enqueue after `ticket`. wrap=False returns only the counts
        (n_episodes, n_records), for a caller that does not read the records."""
        info = HarvestInfo()
        check(lib().bgx_harvest_fetch(self._h, int(ticket), ctypes.byref(info)), "bgx_harvest_fetch")
        if not wrap:
            return int(info.n_episodes), int(info.n_records)
        return self._harvest_from(info, clone)

    def _harvest_from(self, info, clone):
        if info.n_episodes == 0:   # nothing finished: shared empty tensors, no allocation
            if self._empty is None:
                self._empty = Harvest(torch.zeros((0, EP_WORDS), dtype=torch.int32, device=self.device),
                                      torch.zeros((0, REC_WORDS), dtype=torch.int32, device=self.device))
            return self._empty
        hdr = _wrap(info.d_headers, info.n_episodes * EP_WORDS, self.device).view(-1, EP_WORDS)
        rec = _wrap(info.d_records, info.n_records * REC_WORDS, self.device).view(-1, REC_WORDS)
        if clone:
            hdr, rec = hdr.clone(), rec.clone()
        return Harvest(hdr, rec)

    def stats(self):
        s = Stats()
        check(lib().bgx_get_stats(self._h, ctypes.byref(s)), "bgx_get_stats")
        return {k: int(getattr(s, k)) for k, _ in Stats._fields_}

    PEEK = {"lane_rows": (0, "<u4", 8), "player": (1, "u1", 1), "dice": (2, "u1", 2), "cand_off": (3, "<i4", 1),
            "cand_cnt": (4, "<i4", 1), "cand_rows": (5, "<u4", 8), "values": (6, "<f4", 1), "sel": (7, "<i4", 4),
            "job_val": (8, "<f4", 21)}

    def peek(self, name):
        """Test hook (bgx_engine_peek): a host copy of one of the phased
        engine's per-step buffers, e.g. the candidates and the per-(candidate,
        roll) top-5 reply means of the last 2-ply step (include/bgx.h)."""
        import numpy as np
        buf, dt, width = self.PEEK[name]
        n = ctypes.c_uint64(0)
        check(lib().bgx_engine_peek(self._h, buf, None, 0, ctypes.byref(n)), "bgx_engine_peek")
        out = np.empty(int(n.value) // np.dtype(dt).itemsize, dtype=dt)
        check(lib().bgx_engine_peek(self._h, buf, out.ctypes.data_as(ctypes.c_void_p), int(n.value), None),
              "bgx_engine_peek")
        return out.reshape(-1, width) if width > 1 else out

    def set_timing(self, enabled=True):
        check(lib().bgx_set_timing(self._h, 1 if enabled else 0), "bgx_set_timing")

    def timing(self):
        ms_mg, ms_mlp = ctypes.c_double(), ctypes.c_double()
        n_mg, n_mlp = ctypes.c_int(), ctypes.c_int()
        check(lib().bgx_get_timing(self._h, ctypes.byref(ms_mg), ctypes.byref(n_mg), ctypes.byref(ms_mlp),
                                   ctypes.byref(n_mlp)), "bgx_get_timing")
        return {"movegen_ms": ms_mg.value, "movegen_launches": n_mg.value, "mlp_ms": ms_mlp.value,
                "mlp_launches": n_mlp.value}


def _wrap(addr, n, device):
    """Device memory owned by the engine -> torch int32 tensor (no copy)."""
    if n == 0 or not addr:
        return torch.zeros((0,), dtype=torch.int32, device=device)
    # round-trip through the CUDA array interface so torch sees a device buffer
    class _Buf:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<i4", "data": (int(addr), False),
                                    "version": 2, "strides": None}
    return torch.as_tensor(_Buf(), device=device)
