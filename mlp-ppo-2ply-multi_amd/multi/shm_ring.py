"""Shared-memory byte ring for the bulk Episode path.

The reference moves every finished Episode through a multiprocessing.Queue,
i.e. one pickle round trip per episode (~1.5 ms, ~162 KB: src/multi/
experience_queue.py:5-13, src/environments/episode.py:22-46). Workers here
push one message per harvest instead: the compact device records (32-byte
episode headers + 96-byte experience records) copied into a ring in
multiprocessing.shared_memory; the consumer decodes them in bulk.

Layout: a 64-byte control block [write | read | episodes put | messages put |
episodes got | messages got] (i64 each; producers own the "put" words under
the lock, the consumer owns "read" and the "got" words and never takes the
lock, so a producer waiting for space cannot block it), then `capacity` data
bytes. A message is an 8-byte length (with
the episode count in its top 24 bits) followed by the payload, padded to 8
bytes; a length of WRAP means "continue at offset 0". Producers serialise on a
multiprocessing lock and publish by storing the new write offset after the
payload (aligned 8-byte stores; x86-64 keeps store order); the single consumer
publishes consumption the same way. Positions are monotonic byte counts.
"""
from __future__ import annotations

import multiprocessing as mp
import time
from multiprocessing import shared_memory

import numpy as np

CTRL = 64
WRAP = (1 << 40) - 1
LEN_MASK = (1 << 40) - 1


class ShmRing:
    def __init__(self, capacity: int = 256 << 20, lock=None, name: str | None = None):
        self.capacity = (int(capacity) + 7) & ~7
        if name is None:
            self.shm = shared_memory.SharedMemory(create=True, size=CTRL + self.capacity)
            self.owner = True
            self._ctrl()[:] = 0
        else:
            self.shm = shared_memory.SharedMemory(name=name)
            self.owner = False
        self.lock = lock if lock is not None else mp.Lock()
        self._views()

    def _ctrl(self):
        return np.ndarray((8,), dtype=np.int64, buffer=self.shm.buf[:CTRL])

    def _views(self):
        self.ctrl = self._ctrl()
        self.data = np.ndarray((self.capacity,), dtype=np.uint8, buffer=self.shm.buf[CTRL:CTRL + self.capacity])

    # pickling for multiprocessing (spawn): attach by name, share the lock
    def __getstate__(self):
        return {"name": self.shm.name, "capacity": self.capacity, "lock": self.lock}

    def __setstate__(self, st):
        self.capacity = st["capacity"]
        self.lock = st["lock"]
        self.shm = shared_memory.SharedMemory(name=st["name"])
        self.owner = False
        self._views()

    @property
    def pending_episodes(self) -> int:
        return int(self.ctrl[2]) - int(self.ctrl[4])

    @property
    def pending_messages(self) -> int:
        return int(self.ctrl[3]) - int(self.ctrl[5])

    def put(self, payload, n_episodes: int = 0, timeout: float | None = None) -> bool:
        """Append one message (bytes-like). Blocks while the ring is full;
        returns False on timeout. A message larger than the ring raises."""
        buf = np.frombuffer(memoryview(payload).cast("B"), dtype=np.uint8)
        n = buf.size
        need = 8 + ((n + 7) & ~7)
        if need + 8 > self.capacity:
            raise ValueError(f"message of {n} bytes does not fit a ring of {self.capacity} bytes")
        deadline = None if timeout is None else time.monotonic() + timeout
        with self.lock:
            while True:
                w, r = int(self.ctrl[0]), int(self.ctrl[1])
                off = w % self.capacity
                tail = self.capacity - off
                extra = tail if tail < need else 0          # wrap marker + skipped tail
                if self.capacity - (w - r) >= need + extra:
                    break
                if deadline is not None and time.monotonic() > deadline:
                    return False
                time.sleep(0.0005)
            if extra:
                self.data[off:off + 8].view(np.int64)[0] = WRAP
                w += extra
                off = 0
            self.data[off + 8:off + 8 + n] = buf
            self.data[off:off + 8].view(np.int64)[0] = n | (int(n_episodes) << 40)
            self.ctrl[2] += n_episodes
            self.ctrl[3] += 1
            self.ctrl[0] = w + need                          # publish
        return True

    def get(self, timeout: float | None = None):
        """Pop the next message: (payload bytes, n_episodes), or None on timeout.
        Single consumer."""
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            w, r = int(self.ctrl[0]), int(self.ctrl[1])
            if w != r:
                break
            if deadline is not None and time.monotonic() > deadline:
                return None
            time.sleep(0.0005)
        off = r % self.capacity
        word = int(self.data[off:off + 8].view(np.int64)[0])
        if word == WRAP:
            r += self.capacity - off
            off = 0
            word = int(self.data[0:8].view(np.int64)[0])
        n, n_eps = word & LEN_MASK, word >> 40
        payload = self.data[off + 8:off + 8 + n].tobytes()
        self.ctrl[4] += n_eps
        self.ctrl[5] += 1
        self.ctrl[1] = r + 8 + ((n + 7) & ~7)               # release
        return payload, n_eps

    def close(self):
        self.shm.close()
        if self.owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass
