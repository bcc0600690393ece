"""One process per GPU: lane sharding, weight broadcast and episode gather.

The reference moves episodes worker -> trainer through a pickled
multiprocessing.Queue and weights through a Manager dict (src/main.py:65-91,
src/multi/experience_queue.py:5-13, src/multi/parameter_manager.py:79-91).
Here every rank runs its own Engine over a disjoint block of global lane ids
(so results do not depend on the GPU count) and the only collectives are:
  * broadcast_weights  — the 102,404-byte fp32 state on each version bump;
  * gather_episodes    — compact headers (64 B) / records (48 B) of finished
                         episodes to the trainer rank (RCCL point-to-point
                         over xGMI, exact sizes, no padding).
There is no per-step exchange.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .records import EP_WORDS, REC_WORDS

KEYS = ("W1", "b1", "w2", "b2")


def lane_block(rank: int, lanes_per_rank: int):
    """Global lane ids [base, base + lanes) owned by `rank`."""
    return rank * lanes_per_rank, lanes_per_rank


def broadcast_weights(w, src=0, device=None):
    """Broadcast the (W1, b1, w2, b2) fp32 weights from `src`; returns host numpy copies."""
    dev = device or (torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl"
                     else torch.device("cpu"))
    shapes = {"W1": (128, 198), "b1": (128,), "w2": (128,), "b2": (1,)}
    flat = torch.empty(128 * 198 + 128 + 128 + 1, dtype=torch.float32, device=dev)
    if dist.get_rank() == src:
        flat.copy_(torch.from_numpy(np.concatenate([np.asarray(w[k], np.float32).reshape(-1) for k in KEYS])))
    dist.broadcast(flat, src=src)
    out, o = {}, 0
    host = flat.cpu().numpy()
    for k in KEYS:
        n = int(np.prod(shapes[k]))
        out[k] = host[o:o + n].reshape(shapes[k]).copy()
        o += n
    return out


class PendingGather:
    """An episode gather in flight (gather_episodes(..., async_op=True)):
    wait() returns what the synchronous call returns. The buffers stay
    referenced until then."""

    def __init__(self, works, refs, result):
        self._works, self._refs, self._result = works, refs, result

    def wait(self):
        for w in self._works:
            w.wait()
        self._works, self._refs = [], None
        return self._result


def gather_episodes(h, dst=0, keep=False, async_op=False):
    """Gather a Harvest (headers [n, 16], records [m, 12]) from every rank to `dst`.

    Two steps: the per-rank counts go to dst (one 16-byte gather), then each
    rank with episodes sends exactly its headers and records to dst by
    point-to-point send / recv (RCCL over xGMI with the nccl backend; no
    padding to the largest rank, nothing sent by a rank with no episodes).
    Returns (total_episodes, total_records) on dst ((0, 0) elsewhere); with
    keep=True also the per-rank (headers, records) list on dst. With
    async_op=True the point-to-point transfers are left in flight and a
    PendingGather is returned (the counts step is synchronous): the caller's
    next engine steps overlap the transfer."""
    world, rank = dist.get_world_size(), dist.get_rank()
    nccl = dist.get_backend() == "nccl"
    dev = h.headers.device if nccl else torch.device("cpu")
    cnt = torch.tensor([h.n_episodes, h.n_records], dtype=torch.int64, device=dev)
    if rank == dst:
        cnts_t = [torch.zeros_like(cnt) for _ in range(world)]
        dist.gather(cnt, cnts_t, dst=dst)
        cnts = [tuple(int(x) for x in c.tolist()) for c in cnts_t]
    else:
        dist.gather(cnt, None, dst=dst)
        cnts = None
    ops, refs = [], []
    if rank == dst:
        parts = []
        for r in range(world):
            ne, nr = cnts[r]
            if r == dst:
                parts.append((h.headers.to(dev), h.records.to(dev)))
                continue
            hb = torch.empty((ne, EP_WORDS), dtype=torch.int32, device=dev)
            rb = torch.empty((nr, REC_WORDS), dtype=torch.int32, device=dev)
            if ne:
                ops.append(dist.P2POp(dist.irecv, hb, r))
            if nr:
                ops.append(dist.P2POp(dist.irecv, rb, r))
            parts.append((hb, rb))
            refs += [hb, rb]
        tot = (sum(c[0] for c in cnts), sum(c[1] for c in cnts))
        result = (tot[0], tot[1], parts) if keep else tot
    else:
        hs, rs = h.headers.to(dev).contiguous(), h.records.to(dev).contiguous()
        if h.n_episodes:
            ops.append(dist.P2POp(dist.isend, hs, dst))
        if h.n_records:
            ops.append(dist.P2POp(dist.isend, rs, dst))
        refs += [hs, rs]
        result = (0, 0, []) if keep else (0, 0)
    works = dist.batch_isend_irecv(ops) if ops else []
    if async_op:
        return PendingGather(works, refs, result)
    for w in works:
        w.wait()
    return result
