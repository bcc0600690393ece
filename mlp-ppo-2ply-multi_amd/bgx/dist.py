"""One process per GPU: lane sharding, weight broadcast and episode gather.

The reference moves episodes worker -> trainer through a pickled
multiprocessing.Queue and weights through a Manager dict (src/main.py:65-91,
src/multi/experience_queue.py:5-13, src/multi/parameter_manager.py:79-91).
Here every rank runs its own Engine over a disjoint block of global lane ids
(so results do not depend on the GPU count) and the only collectives are:
  * broadcast_weights  — the 102,404-byte fp32 state on each version bump;
  * gather_episodes    — compact headers/records of finished episodes to the
                         trainer rank (RCCL point-to-point over xGMI).
There is no per-step exchange.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

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


def _pad_rows(t, n, width, device):
    out = torch.zeros((n, width), dtype=torch.int32, device=device)
    if t.shape[0]:
        out[: t.shape[0]] = t
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
    """Gather a Harvest (headers [n, 8], records [m, 24]) from every rank to `dst`.

    Returns (total_episodes, total_records) on dst ((0, 0) elsewhere); with
    keep=True also the per-rank (headers, records) list on dst. With
    async_op=True the two data gathers are left in flight and a PendingGather
    is returned (the counts exchange is still synchronous): the caller's next
    engine steps overlap the transfer."""
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = h.headers.device if dist.get_backend() == "nccl" else torch.device("cpu")
    cnt = torch.tensor([h.n_episodes, h.n_records], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt)
    cnts = [tuple(int(x) for x in c.tolist()) for c in cnts]
    me = max(c[0] for c in cnts)
    mr = max(c[1] for c in cnts)
    hdr = _pad_rows(h.headers.to(dev), max(me, 1), 8, dev)
    rec = _pad_rows(h.records.to(dev), max(mr, 1), 24, dev)
    if rank == dst:
        hl = [torch.empty_like(hdr) for _ in range(world)]
        rl = [torch.empty_like(rec) for _ in range(world)]
        works = [dist.gather(hdr, hl, dst=dst, async_op=async_op), dist.gather(rec, rl, dst=dst, async_op=async_op)]
        parts = [(hl[r][: cnts[r][0]], rl[r][: cnts[r][1]]) for r in range(world)]
        tot = (sum(c[0] for c in cnts), sum(c[1] for c in cnts))
        result = (tot[0], tot[1], parts) if keep else tot
        refs = (hdr, rec, hl, rl)
    else:
        works = [dist.gather(hdr, None, dst=dst, async_op=async_op), dist.gather(rec, None, dst=dst, async_op=async_op)]
        result = (0, 0, []) if keep else (0, 0)
        refs = (hdr, rec)
    return PendingGather(works, refs, result) if async_op else result
