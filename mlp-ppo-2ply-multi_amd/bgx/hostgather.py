"""Episode gather of the ranks of one node over the DMA engines (no kernels,
no collective per harvest).

The reference hands finished episodes from its 7 workers to main.py through a
pickled multiprocessing.Queue (src/main.py:115-133,
src/multi/experience_queue.py:5-13): a host-side hand-off. Here every rank
runs its own Engine on its GPU; after a harvest it copies the compact
headers (64 B) and records (48 B) device -> host straight into a host
segment that is page-locked for DMA (bgx_host_register), on a DMA engine
(bgx_dma_copy_d2h: SDMA through the HSA runtime, so the transfer runs while
the persistent fused kernel holds every compute unit; the HIP runtime here
would serve hipMemcpyAsync with a blit kernel, which waits for free compute
units — BGX_HG_COPY=hip selects that path). The counts travel in the same
segment: there is no per-harvest collective. The trainer rank reads every
peer's batch from host memory (where main.py's consumer wants them) and
acknowledges it.

Segments are anonymous memory files (memfd_create), not /dev/shm files: a
container's /dev/shm is often a 64 MB tmpfs, while a rank's segment is
~0.5 GB at 8,192 lanes, and a tmpfs accepts a larger file and fails only when
its pages are touched. A memfd is limited by the host's memory alone. Each
rank creates its own; the trainer rank receives the peers' descriptors once,
at setup, over a Unix socket (SCM_RIGHTS) and maps them. So the host path
has no capacity-dependent fallback: bench.py --gpus N takes it whatever
/dev/shm holds (tests/test_gpu_dist.py runs it with two ranks on one GPU).

Protocol (per rank r != dst, batch numbers 1, 2, ... ; two slots):
  publish(h): wait until dst acknowledged batch seq - 2 (the slot's previous
              batch), enqueue the two copies into slot seq % 2, return a
              Pending; Pending.wait() waits for the copies, then stores the
              counts and finally the batch number (the store that publishes).
  collect(seq) on dst: for every peer, wait until its published number
              reaches seq, read counts and data, store the acknowledgement.
A rank can run at most one batch ahead of dst's reads; nothing else couples
the ranks. Segment header (i64): [0] published batch, [1 + 2 s] episodes and
[2 + 2 s] records of the batch in slot s, [5] acknowledged batch (written by
dst). The counts are per slot: a rank one batch ahead rewrites only its
other slot's.
"""
from __future__ import annotations

import mmap
import os
import secrets
import socket
import time

import numpy as np
import torch

from .records import EP_WORDS, REC_WORDS

HDR = 64
EP_BYTES, REC_BYTES = EP_WORDS * 4, REC_WORDS * 4
COPY_KIND = int(os.environ.get("BGX_HG_COPY_KIND", "2"))   # bgx_copy_async kind: 2 = device -> host


def slot_bytes_for(lanes: int, steps_per_harvest: int, max_steps: int = 300) -> int:
    """A harvest holds at most one record per lane-step since the last one,
    plus the not yet harvested part of every lane's current episode, and at
    most one header per 13 lane-steps (the shortest game) + one per lane."""
    recs = lanes * (steps_per_harvest + max_steps)
    eps = lanes * (steps_per_harvest // 13 + 2)
    return ((recs * REC_BYTES + eps * EP_BYTES) + 4095) & ~4095


# batches whose DMA copy did not finish within its timeout: kept referenced (with
# their source arrays) for the life of the process, since the engine may still
# read and write their memory (bgx_dma_wait leaves such a copy in flight)
STUCK_COPIES = []


class Pending:
    """A batch in flight. It holds the source arrays (`keep`) until wait()
    has seen the copies finish: the caller may drop its Harvest at once, and
    the caching allocator cannot hand the blocks to anything else while a DMA
    engine still reads them."""

    def __init__(self, gather, seq, n_eps, n_recs, slot, event, dma=(), keep=None):
        self.g, self.seq, self.n_eps, self.n_recs, self.slot, self.event = gather, seq, n_eps, n_recs, slot, event
        self.dma = dma
        self.keep = keep
        self.done = False
        gather.open_batch = self

    def wait(self):
        if self.event is not None:
            self.event.synchronize()
        if self.dma:
            from ._lib import BgxError, check, lib
            for i, t in enumerate(self.dma):
                try:
                    check(lib().bgx_dma_wait(t, int(self.g.timeout * 1000)), "bgx_dma_wait")
                except BgxError:
                    # the copy may still be running: its source blocks and the
                    # destination slot stay owned by it for the life of the
                    # process, and the gather refuses further batches
                    self.dma = self.dma[i:]
                    STUCK_COPIES.append(self)
                    self.g.broken = True
                    raise
            self.dma = ()
        self.keep = None
        c = self.g.ctrl[self.g.rank]
        c[1 + 2 * self.slot], c[2 + 2 * self.slot] = self.n_eps, self.n_recs
        c[0] = self.seq            # publishes (aligned 8-byte store after the counts)
        self.done = True
        return self.seq


class _Segment:
    """An anonymous shared memory file (memfd) mapped into this process."""

    def __init__(self, name, size=None, fd=None):
        if fd is None:
            fd = os.memfd_create(name, os.MFD_CLOEXEC)
            os.ftruncate(fd, size)
        else:
            size = os.fstat(fd).st_size
        self.fd, self.size = fd, size
        self.mm = mmap.mmap(fd, size, flags=mmap.MAP_SHARED, prot=mmap.PROT_READ | mmap.PROT_WRITE)
        self.buf = memoryview(self.mm)

    def close(self):
        # (views a caller still holds keep the mapping; it goes with the process)
        for f in (self.buf.release, self.mm.close):
            try:
                f()
            except (BufferError, ValueError):
                pass
        try:
            os.close(self.fd)
        except OSError:
            pass


class HostGather:
    """One per rank. `tag` names the segments (every rank must pass the same
    one, e.g. from make_tag()); slot_bytes from slot_bytes_for()."""

    def __init__(self, rank: int, world: int, tag: str, slot_bytes: int, dst: int = 0, device=None,
                 timeout: float = 120.0):
        self.rank, self.world, self.dst, self.tag = rank, world, dst, tag
        self.slot_bytes = int(slot_bytes)
        self.timeout = timeout
        self.device = device
        self.seq = 0
        self.open_batch = None   # the last Pending: a batch is published by its wait(), before the next one
        self.broken = False   # a DMA copy of this gather timed out (Pending.wait): no further batches
        self._mine = _Segment(self._name(rank), size=HDR + 2 * self.slot_bytes)
        self.shm = {rank: self._mine}
        np.ndarray((8,), np.int64, buffer=self._mine.buf[:HDR])[:] = 0
        self.ctrl = {rank: np.ndarray((8,), np.int64, buffer=self._mine.buf[:HDR])}
        self._registered = None
        self._stream = None
        # device -> host path: "dma" (bgx_dma_copy_d2h, SDMA engine) or "hip"
        # (hipMemcpyAsync on a side stream: a blit kernel on this ROCm)
        self.copy = os.environ.get("BGX_HG_COPY", "dma")
        if device is not None and torch.cuda.is_available():
            from ._lib import check, lib
            addr = np.frombuffer(self._mine.buf, np.uint8).ctypes.data
            check(lib().bgx_host_register(addr, HDR + 2 * self.slot_bytes), "bgx_host_register")
            self._registered = addr
            self._stream = torch.cuda.Stream(device=device)

    def _name(self, r):
        return f"bgx_hg_{self.tag}_{r}"

    def _sock_name(self):
        return f"\0{self._name('dst')}".encode()

    def listen(self):
        """dst, before the peers connect: the socket that receives their segments."""
        if self.rank != self.dst:
            return
        self._listener = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self._listener.bind(self._sock_name())   # abstract namespace: no file, no /dev/shm
        self._listener.listen(self.world)

    def send_segment(self):
        """Rank != dst: hand this rank's segment descriptor to dst (SCM_RIGHTS)."""
        if self.rank == self.dst:
            return
        with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as so:
            so.settimeout(self.timeout)
            so.connect(self._sock_name())
            socket.send_fds(so, [int(self.rank).to_bytes(4, "little")], [self._mine.fd])
            so.recv(1)   # dst has mapped it

    def attach(self):
        """dst: receive and map every peer's segment (after listen())."""
        if self.rank != self.dst:
            return
        self._listener.settimeout(self.timeout)
        for _ in range(self.world - 1):
            conn, _addr = self._listener.accept()
            with conn:
                msg, fds, _flags, _addr = socket.recv_fds(conn, 4, 1)
                r = int.from_bytes(msg, "little")
                s = _Segment(None, fd=fds[0])
                self.shm[r] = s
                self.ctrl[r] = np.ndarray((8,), np.int64, buffer=s.buf[:HDR])
                conn.sendall(b"k")
        self._listener.close()

    def _slot(self, r, slot):
        base = HDR + slot * self.slot_bytes
        return self.shm[r].buf[base:base + self.slot_bytes]

    def _spin(self, cond, what):
        # poll without sleeping for the first 2 ms (a peer's batch lands ~0.1-1 ms
        # after its harvest; a 0.2 ms sleep would add up to that much to the
        # hand-off), then back off
        t0 = time.monotonic()
        while not cond():
            el = time.monotonic() - t0
            if el > self.timeout:
                raise TimeoutError(f"HostGather rank {self.rank}: {what}")
            if el > 0.002:
                time.sleep(0.0002)

    def publish(self, h, ready: bool = False) -> Pending:
        """Rank != dst: start the copy of a Harvest into this rank's segment.
        ready=True: the harvest's device arrays are complete (bgx_harvest_fetch
        waited for them); otherwise the current stream is synchronized first."""
        n_eps, n_recs = h.n_episodes, h.n_records
        if self.broken:
            raise RuntimeError("HostGather: an earlier DMA copy did not finish; its slot is still owned by it")
        if self.open_batch is not None and not self.open_batch.done:
            # publishing c[0] = seq + 1 first would make dst read batch seq's slot
            # with the counts of the batch before it
            raise RuntimeError(f"HostGather: batch {self.open_batch.seq} was not waited for before the next publish")
        need = n_eps * EP_BYTES + n_recs * REC_BYTES
        if need > self.slot_bytes:   # before the batch number moves: dst still waits for the same batch
            raise ValueError(f"harvest of {need} bytes > slot of {self.slot_bytes} (slot_bytes_for)")
        self.seq += 1
        seq, slot = self.seq, self.seq % 2
        c = self.ctrl[self.rank]
        self._spin(lambda: int(c[5]) >= seq - 2, f"dst did not read batch {seq - 2}")
        dst = np.frombuffer(self._slot(self.rank, slot), np.uint8)
        if n_eps == 0:
            return Pending(self, seq, 0, 0, slot, None)
        if h.headers.is_cuda and self._stream is not None and self.copy == "dma":
            # DMA engine (bgx_dma_copy_d2h): the copy runs beside a persistent kernel
            import ctypes
            from ._lib import check, lib
            if not ready:
                torch.cuda.current_stream(h.headers.device).synchronize()
            base = dst.ctypes.data
            t1, t2 = ctypes.c_uint64(0), ctypes.c_uint64(0)
            dev = h.headers.device.index
            check(lib().bgx_dma_copy_d2h(base, h.headers.data_ptr(), n_eps * EP_BYTES, dev, ctypes.byref(t1)),
                  "bgx_dma_copy_d2h")
            check(lib().bgx_dma_copy_d2h(base + n_eps * EP_BYTES, h.records.data_ptr(), n_recs * REC_BYTES, dev,
                                         ctypes.byref(t2)), "bgx_dma_copy_d2h")
            return Pending(self, seq, n_eps, n_recs, slot, None, dma=(t1.value, t2.value),
                           keep=(h.headers, h.records))
        if h.headers.is_cuda and self._stream is not None:
            from ._lib import check, lib
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(h.headers.device))
            self._stream.wait_event(ev)
            # the side stream reads the arrays: the allocator must not reuse them before it is done
            h.headers.record_stream(self._stream)
            h.records.record_stream(self._stream)
            base = dst.ctypes.data
            s = self._stream.cuda_stream
            check(lib().bgx_copy_async(base, h.headers.data_ptr(), n_eps * EP_BYTES, COPY_KIND, s),
                  "bgx_copy_async")
            check(lib().bgx_copy_async(base + n_eps * EP_BYTES, h.records.data_ptr(), n_recs * REC_BYTES, COPY_KIND,
                                       s), "bgx_copy_async")
            done = torch.cuda.Event()
            done.record(self._stream)
            # the engine's buffers must outlive the copy: the caller waits this
            # Pending before its next harvest (bgx_harvest reuses them)
            return Pending(self, seq, n_eps, n_recs, slot, done, keep=(h.headers, h.records))
        hb = h.headers.cpu().numpy().view(np.uint8).reshape(-1)
        rb = h.records.cpu().numpy().view(np.uint8).reshape(-1)
        dst[:hb.size] = hb
        dst[hb.size:hb.size + rb.size] = rb
        return Pending(self, seq, n_eps, n_recs, slot, None)

    def collect(self, seq: int, copy: bool = True):
        """dst: every peer's batch `seq` as (headers uint32 [n, 16], records
        uint32 [m, 12]) host arrays, in rank order (dst's own entry is None:
        the caller has its harvest). copy=False returns views that stay valid
        until the peer reuses the slot (two batches later)."""
        out = []
        for r in range(self.world):
            if r == self.dst:
                out.append(None)
                continue
            c = self.ctrl[r]
            self._spin(lambda: int(c[0]) >= seq, f"rank {r} did not publish batch {seq}")
            slot = seq % 2
            n_eps, n_recs = int(c[1 + 2 * slot]), int(c[2 + 2 * slot])
            raw = np.frombuffer(self._slot(r, slot), np.uint8)
            hdr = raw[:n_eps * EP_BYTES].view(np.uint32).reshape(-1, EP_WORDS)
            rec = raw[n_eps * EP_BYTES:n_eps * EP_BYTES + n_recs * REC_BYTES].view(np.uint32).reshape(-1, REC_WORDS)
            if copy:
                hdr, rec = hdr.copy(), rec.copy()
            out.append((hdr, rec))
            if copy:
                c[5] = seq      # acknowledged: the peer may reuse this slot
        return out

    def ack(self, seq: int):
        """dst, after collect(seq, copy=False): release every peer's slot."""
        for r in range(self.world):
            if r != self.dst:
                self.ctrl[r][5] = seq

    def close(self):
        if self._registered is not None:
            from ._lib import lib
            lib().bgx_host_unregister(self._registered)
            self._registered = None
        self.ctrl = {}
        for s in list(self.shm.values()):
            s.close()
        self.shm = {}
        lst = getattr(self, "_listener", None)
        if lst is not None:
            lst.close()


def make_tag() -> str:
    """A fresh segment tag (rank 0 makes it; broadcast it to the others)."""
    return f"{os.getpid()}_{secrets.token_hex(4)}"


def setup(rank: int, world: int, slot_bytes: int, dst: int = 0, device=None, timeout=None) -> HostGather:
    """Collective once (torch.distributed): agree on a tag, create the
    segments, hand their descriptors to dst. No collective afterwards."""
    import torch.distributed as dist
    obj = [make_tag() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    if timeout is None:   # seconds a rank waits for a peer before it fails (BGX_GATHER_TIMEOUT)
        timeout = float(os.environ.get("BGX_GATHER_TIMEOUT", "120"))
    g = HostGather(rank, world, obj[0], slot_bytes, dst=dst, device=device, timeout=timeout)
    g.listen()
    dist.barrier()
    g.send_segment()
    g.attach()
    dist.barrier()
    return g
