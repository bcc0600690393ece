"""Harvest device -> host on a DMA engine, into a page-locked staging buffer.

On this ROCm a device -> host torch copy (`tensor.cpu()`) is served by a blit
kernel, which needs compute units: behind a queued persistent fused launch it
waits for that launch to end, so a worker that copies its previous harvest
while the next launch runs would stall the GPU for its host work every cycle.
bgx_dma_copy_d2h (SDMA through the HSA runtime) runs beside the launch
instead. One Staging per engine: the returned arrays are views into the
buffer, valid until the next copy.
"""
from __future__ import annotations

import ctypes
import mmap

import numpy as np

from .records import EP_WORDS, REC_WORDS


class Staging:
    def __init__(self, device: int):
        self.device = device
        self.size = 0
        self.mm = None
        self.buf = None
        self.addr = None
        self.broken = False   # a copy timed out (copy()): its buffer is never reused

    def _ensure(self, nbytes: int):
        if nbytes <= self.size:
            return
        from ._lib import check, lib
        self.close()
        size = max(1 << 20, (nbytes * 5 // 4 + 4095) & ~4095)
        self.mm = mmap.mmap(-1, size)   # anonymous, page-aligned
        self.buf = np.frombuffer(self.mm, np.uint8)
        self.addr = self.buf.ctypes.data
        check(lib().bgx_host_register(self.addr, size), "bgx_host_register")
        self.size = size

    def copy(self, h, timeout_ms: int = 60000):
        """(headers uint32 [n, 16], records uint32 [m, 12]) of a Harvest whose
        device arrays are complete (harvest_fetch waited for them)."""
        from ._lib import check, lib
        if self.broken:
            raise RuntimeError("Staging: an earlier DMA copy did not finish; its buffer is still owned by it")
        ne, nr = h.n_episodes, h.n_records
        hb, rb = ne * EP_WORDS * 4, nr * REC_WORDS * 4
        if ne == 0:
            return np.zeros((0, EP_WORDS), np.uint32), np.zeros((0, REC_WORDS), np.uint32)
        self._ensure(hb + rb)
        t1, t2 = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(lib().bgx_dma_copy_d2h(self.addr, h.headers.data_ptr(), hb, self.device, ctypes.byref(t1)),
              "bgx_dma_copy_d2h")
        check(lib().bgx_dma_copy_d2h(self.addr + hb, h.records.data_ptr(), rb, self.device, ctypes.byref(t2)),
              "bgx_dma_copy_d2h")
        from ._lib import BgxError
        tickets = [t1.value, t2.value]
        try:
            while tickets:
                check(lib().bgx_dma_wait(tickets[0], timeout_ms), "bgx_dma_wait")
                tickets.pop(0)   # released by the successful wait
        except BgxError:
            # a copy still in flight owns the staging buffer and the harvest's
            # arrays: keep both for the life of the process, with the tickets not
            # yet waited for (each still holds its completion signal; a later
            # bgx_dma_wait on one of them releases it), and refuse further copies
            from .hostgather import STUCK_COPIES
            STUCK_COPIES.append((self.mm, self.buf, h, tuple(tickets)))
            self.mm = self.buf = self.addr = None
            self.size = 0
            self.broken = True
            raise
        hdr = self.buf[:hb].view(np.uint32).reshape(ne, EP_WORDS)
        rec = self.buf[hb:hb + rb].view(np.uint32).reshape(nr, REC_WORDS)
        return hdr, rec

    def close(self):
        if self.addr is not None:
            from ._lib import lib
            lib().bgx_host_unregister(self.addr)
            self.addr = None
        self.buf = None
        if self.mm is not None:
            try:
                self.mm.close()
            except BufferError:
                pass   # a caller still holds a view; the mapping goes with the process
            self.mm = None
        self.size = 0
