"""Workload for the copy-engine overlap trace: one
engine at 8,192 lanes (balanced fused launches), each harvest handed to a
HostGather segment by the DMA engines (bgx_copy_async on a side stream)
while the next fused launch runs -- bench.py --gather host's data path on one
GPU. Run it under
  rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o run --output-format csv -- python tools/overlap_probe.py
and check the spans with tools/overlap_check.py DIR. Development tool."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx import Engine, hostgather  # noqa: E402

d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
w = {k: d[k] for k in ("W1", "b1", "w2", "b2")}
lanes, chunk = 8192, int(os.environ.get("CHUNK", "100"))
torch.cuda.set_device(0)
e = Engine(lanes=lanes, seed=3, balance=True)
e.set_weights(w, 1.5, 1)
e.step(300)
e.harvest()
# a one-rank stand-in for a peer: this process publishes (rank 1) and reads its own segment as dst
g = hostgather.HostGather(1, 2, hostgather.make_tag(), hostgather.slot_bytes_for(lanes, chunk), dst=1, device=0)
pend_t, inflight, n_bytes = None, None, 0
for i in range(12):
    if inflight is not None:
        inflight.wait()
        g.ctrl[1][5] = inflight.seq          # acknowledge (the reader's store)
    e.step(chunk)
    t = e.harvest_enqueue()
    if pend_t is not None:
        h = e.harvest_fetch(pend_t)
        n_bytes += h.n_episodes * 64 + h.n_records * 48
        inflight = g.publish(h, ready=True)  # DMA copy, concurrent with the launch just queued
    pend_t = t
if inflight is not None:
    inflight.wait()
torch.cuda.synchronize()
print(f"overlap probe: 12 launches of {chunk} steps, {n_bytes / 1e6:.1f} MB copied device -> shared host memory")
g.close()
e.close()
