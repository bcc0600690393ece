"""ExperienceQueue (src/multi/experience_queue.py:5-13) with a bulk path.

Reference surface: put(episode), get(timeout) (raises queue.Empty), qsize().
Episodes put one by one still travel through a multiprocessing.Queue. The
bulk path: a worker calls put_records(headers, records)
once per harvest with the engine's compact records (EP_WORDS / REC_WORDS
uint32 words per episode / experience); they go through a shared-memory ring
(multi/shm_ring.py) instead of one pickle per episode, and get() decodes a
whole message at once on the GPU (bgx_unpack + bgx_encode_packed for the 198-d
observations) before handing out Episodes one at a time, so src/main.py's
`q.get(timeout=1)` loop runs unchanged.

BGX_QUEUE_MB (256) sizes the ring.
"""
from __future__ import annotations

import collections
import multiprocessing as mp
import os
import queue
import time

import numpy as np

from .shm_ring import ShmRing

from bgx.records import EP_WORDS, REC_WORDS  # noqa: E402  (the engine's wire format)


def pack_message(headers: np.ndarray, records: np.ndarray) -> bytes:
    h = np.ascontiguousarray(headers, dtype=np.uint32).reshape(-1, EP_WORDS)
    r = np.ascontiguousarray(records, dtype=np.uint32).reshape(-1, REC_WORDS)
    return np.array([h.shape[0], r.shape[0]], np.uint32).tobytes() + h.tobytes() + r.tobytes()


def unpack_message(payload: bytes):
    a = np.frombuffer(payload, dtype=np.uint32)
    ne, nr = int(a[0]), int(a[1])
    h = a[2:2 + ne * EP_WORDS].reshape(ne, EP_WORDS)
    r = a[2 + ne * EP_WORDS:2 + ne * EP_WORDS + nr * REC_WORDS].reshape(nr, REC_WORDS)
    return h, r


class ExperienceQueue:
    def __init__(self, capacity_mb: int | None = None, ctx=None):
        # ctx: the multiprocessing context the workers are started with (default:
        # the current default, which src/main.py:164 sets to "spawn")
        ctx = ctx if ctx is not None else mp.get_context()
        self.queue = ctx.Queue()
        mb = capacity_mb if capacity_mb is not None else int(os.environ.get("BGX_QUEUE_MB", "256"))
        self.ring = ShmRing(mb << 20, lock=ctx.Lock())
        self._ready = collections.deque()

    def __getstate__(self):
        return {"queue": self.queue, "ring": self.ring}

    def __setstate__(self, st):
        self.queue = st["queue"]
        self.ring = st["ring"]
        self._ready = collections.deque()

    # --- reference surface
    def put(self, episode):
        self.queue.put(episode)

    def get(self, timeout=None):
        if self._ready:
            return self._ready.popleft()
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            try:
                return self.queue.get_nowait()
            except queue.Empty:
                pass
            msg = self.ring.get(timeout=0.001)
            if msg is not None:
                eps = self._decode(msg[0])
                if eps:
                    self._ready.extend(eps[1:])
                    return eps[0]
            if deadline is not None and time.monotonic() > deadline:
                raise queue.Empty

    def qsize(self):
        try:
            q = self.queue.qsize()
        except NotImplementedError:   # macOS
            q = 0
        return q + len(self._ready) + self.ring.pending_episodes

    # --- bulk path
    def put_records(self, headers, records, timeout=None) -> bool:
        """One harvest (host arrays: headers [n, 16], records [m, 12] uint32, the
        episodes' records contiguous in header order) as one ring message."""
        h = np.asarray(headers)
        return self.ring.put(pack_message(h, records), n_episodes=int(h.shape[0]), timeout=timeout)

    def get_records(self, timeout=None):
        """Raw bulk access for a batch consumer (e.g. a device trainer):
        (headers, records) numpy views of the next message, or None."""
        msg = self.ring.get(timeout=timeout)
        return None if msg is None else unpack_message(msg[0])

    def _decode(self, payload):
        import torch   # the consumer decodes on its GPU (bgx kernels), like the worker would

        from bgx.episodes import episodes_from_arrays
        from environments import Episode, Experience, Player
        h, r = unpack_message(payload)
        rec = torch.from_numpy(r.view(np.int32).copy()).cuda()
        return episodes_from_arrays(h, rec, Episode, Experience, Player)

    def close(self):
        self.ring.close()
