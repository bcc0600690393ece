"""Episode gather straight into the trainer rank's GPU memory (xGMI peer
copies on the source GPUs' DMA engines; no kernels, no collective per
harvest).

The reference's consumer takes each Episode from the queue and moves it to
the trainer's device (src/main.py:115-133: `q.get()`, `episode.to_tensor(
device)`, `Trainer.update`). bgx/hostgather.py lands the ranks' harvests in
host memory, so a GPU trainer (bgx.trainer.DeviceTrainer, bgx_td0_update)
would copy every record host -> device again. Here the trainer rank (dst)
allocates, on its GPU, two slots per peer rank; each peer opens that
allocation once (bgx_ipc_open: inter-process access to device memory, one
process per GPU) and after a harvest copies its compact headers (64 B) and
records (48 B) device -> device into its slot with bgx_dma_copy_d2d (an SDMA
engine of the peer's GPU; over xGMI between two GPUs, within one GPU when
ranks share it, as in tests/test_gpu_dist.py). The counts and the batch number
travel through the host control words of bgx/hostgather.py (same protocol:
two slots per rank, a rank at most one batch ahead of dst's reads), so dst
sees a batch complete only after its copies have finished. collect() returns
device tensors on dst's GPU: the records go to DeviceTrainer.update_records
without touching host memory.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from .hostgather import EP_BYTES, REC_BYTES, HostGather, Pending, make_tag, slot_bytes_for  # noqa: F401
from .records import EP_WORDS, REC_WORDS


def pci_location(index: int):
    """(PCI domain, bus, device) of this process's GPU `index`."""
    p = torch.cuda.get_device_properties(index)
    return int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)


def device_by_pci(loc) -> int:
    """This process's ordinal of the GPU at PCI location `loc`."""
    loc = tuple(int(x) for x in loc)
    for i in range(torch.cuda.device_count()):
        if pci_location(i) == loc:
            return i
    raise RuntimeError(f"DeviceGather: the trainer rank's GPU (PCI {loc[0]:04x}:{loc[1]:02x}:{loc[2]:02x}) is not "
                       "visible to this process (HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES): a peer copy needs it")


class DeviceGather(HostGather):
    """One per rank. dst holds the slots ([world][2][slot_bytes] on its GPU);
    the control words are HostGather's header-only segments."""

    def __init__(self, rank: int, world: int, tag: str, slot_bytes: int, dst: int = 0, device=None,
                 timeout: float = 120.0):
        super().__init__(rank, world, tag, 0, dst=dst, device=None, timeout=timeout)
        self.slot_bytes = int(slot_bytes)
        self.device = torch.device(device if device is not None else "cuda")
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.buf = None          # dst: the slots
        self.remote = None       # peers: dst's slots opened in this process
        self.remote_off = 0
        self.dst_dev = None
        if rank == dst:
            self.buf = torch.empty(world * 2 * self.slot_bytes, dtype=torch.uint8, device=self.device)

    # ---- setup (collective once, see setup())
    def export(self):
        """dst: (IPC handle, offset, PCI location of dst's GPU) of its slots. The
        GPU travels as its PCI (domain, bus, device), not as an ordinal: an
        ordinal names the same GPU in two processes only when both see the
        same device list (per-rank HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES
        renumber it)."""
        from ._lib import check, lib
        h = (ctypes.c_uint8 * 64)()
        off = ctypes.c_uint64(0)
        check(lib().bgx_ipc_export(self.buf.data_ptr(), h, ctypes.byref(off)), "bgx_ipc_export")
        return bytes(h), int(off.value), pci_location(self.dev_index)

    def open(self, info):
        """Peer: map dst's slots into this process; dst's GPU is found in this
        process's device list by its PCI location."""
        from ._lib import check, lib
        handle, off, loc = info
        dst_dev = device_by_pci(loc)
        with torch.cuda.device(self.device):
            p = ctypes.c_void_p(0)
            check(lib().bgx_ipc_open((ctypes.c_uint8 * 64).from_buffer_copy(handle), off, ctypes.byref(p)),
                  "bgx_ipc_open")
        self.remote, self.remote_off, self.dst_dev = int(p.value), off, int(dst_dev)

    def _slot_off(self, r, slot):
        return (2 * r + slot) * self.slot_bytes

    # ---- data path
    def publish(self, h, ready: bool = False) -> Pending:
        """Rank != dst: start the device -> device copies of a Harvest into its
        slot on dst's GPU (ready: as HostGather.publish)."""
        from ._lib import check, lib
        n_eps, n_recs = h.n_episodes, h.n_records
        if self.broken:
            raise RuntimeError("DeviceGather: an earlier DMA copy did not finish; its slot is still owned by it")
        if self.open_batch is not None and not self.open_batch.done:
            raise RuntimeError(f"DeviceGather: batch {self.open_batch.seq} was not waited for before the next publish")
        need = n_eps * EP_BYTES + n_recs * REC_BYTES
        if need > self.slot_bytes:   # before the batch number moves: dst still waits for the same batch
            raise ValueError(f"harvest of {need} bytes > slot of {self.slot_bytes} (slot_bytes_for)")
        self.seq += 1
        seq, slot = self.seq, self.seq % 2
        c = self.ctrl[self.rank]
        self._spin(lambda: int(c[5]) >= seq - 2, f"dst did not read batch {seq - 2}")
        if n_eps == 0:
            return Pending(self, seq, 0, 0, slot, None)
        if not ready:
            torch.cuda.current_stream(h.headers.device).synchronize()
        base = self.remote + self._slot_off(self.rank, slot)
        src_dev = h.headers.device.index
        t1, t2 = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(lib().bgx_dma_copy_d2d(base, self.dst_dev, h.headers.data_ptr(), src_dev, n_eps * EP_BYTES,
                                     ctypes.byref(t1)), "bgx_dma_copy_d2d")
        check(lib().bgx_dma_copy_d2d(base + n_eps * EP_BYTES, self.dst_dev, h.records.data_ptr(), src_dev,
                                     n_recs * REC_BYTES, ctypes.byref(t2)), "bgx_dma_copy_d2d")
        return Pending(self, seq, n_eps, n_recs, slot, None, dma=(t1.value, t2.value), keep=(h.headers, h.records))

    def collect(self, seq: int, copy: bool = True):
        """dst: every peer's batch `seq` as (headers uint32 [n, 16], records
        uint32 [m, 12]) tensors on dst's GPU, in rank order (dst's own entry is
        None). copy=False: views valid until the peer reuses the slot (call
        ack(seq) when done)."""
        out = []
        for r in range(self.world):
            if r == self.dst:
                out.append(None)
                continue
            c = self.ctrl[r]
            self._spin(lambda: int(c[0]) >= seq, f"rank {r} did not publish batch {seq}")
            slot = seq % 2
            n_eps, n_recs = int(c[1 + 2 * slot]), int(c[2 + 2 * slot])
            o = self._slot_off(r, slot)
            raw = self.buf[o:o + n_eps * EP_BYTES + n_recs * REC_BYTES]
            hdr = raw[:n_eps * EP_BYTES].view(torch.int32).view(-1, EP_WORDS)
            rec = raw[n_eps * EP_BYTES:].view(torch.int32).view(-1, REC_WORDS)
            if copy:
                with torch.cuda.device(self.device):
                    hdr, rec = hdr.clone(), rec.clone()
            out.append((hdr, rec))
        if copy:
            # the clones run on dst's current stream, possibly queued behind its own
            # persistent launch: they must have READ the slots before a peer is told
            # it may overwrite them (its next publish is an SDMA write into the slot)
            torch.cuda.current_stream(self.device).synchronize()
            for r in range(self.world):
                if r != self.dst:
                    self.ctrl[r][5] = seq   # acknowledged: the peer may reuse this slot
        return out

    def close(self):
        if self.remote is not None:
            from ._lib import lib
            lib().bgx_ipc_close(self.remote, self.remote_off)
            self.remote = None
        self.buf = None
        super().close()


def setup(rank: int, world: int, slot_bytes: int, dst: int = 0, device=None, timeout=None) -> DeviceGather:
    """Collective once (torch.distributed): the control segments as
    hostgather.setup, then dst's slots exported and opened by every peer."""
    import torch.distributed as dist
    obj = [make_tag() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    if timeout is None:   # seconds a rank waits for a peer before it fails (BGX_GATHER_TIMEOUT)
        timeout = float(os.environ.get("BGX_GATHER_TIMEOUT", "120"))
    g = DeviceGather(rank, world, obj[0], slot_bytes, dst=dst, device=device, timeout=timeout)
    g.listen()
    dist.barrier()
    g.send_segment()
    g.attach()
    info = [g.export() if rank == dst else None]
    dist.broadcast_object_list(info, src=dst)
    if rank != dst:
        g.open(info[0])
    dist.barrier()
    return g


def as_numpy(batch):
    """collect()'s device tensors -> host uint32 arrays (tests, host consumers)."""
    return [None if b is None else (b[0].cpu().numpy().view(np.uint32), b[1].cpu().numpy().view(np.uint32))
            for b in batch]
