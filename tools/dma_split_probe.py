"""bgx_dma_copy_d2h of harvest-sized buffers (2, 8, 32 MiB) into a page-locked
shared-memory segment, split over BGX_DMA_ENGINES SDMA engines (set by the
caller; read once per process): host-timed median of 10 copies and a content
check. Development tool."""
import ctypes
import json
import os
import sys
import time
from multiprocessing import shared_memory

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx._lib import check, lib  # noqa: E402

N = 32 << 20
dev = torch.arange(N // 4, dtype=torch.int32, device="cuda")
shm = shared_memory.SharedMemory(create=True, size=N)
addr = np.frombuffer(shm.buf, np.uint8).ctypes.data
check(lib().bgx_host_register(addr, N), "register")
torch.cuda.synchronize()
out = {"engines_env": os.environ.get("BGX_DMA_ENGINES", "all")}
for mb in (2, 8, 32):
    n = mb << 20
    ts = []
    for _ in range(10):
        np.frombuffer(shm.buf, np.uint8)[:n] = 0
        tk = ctypes.c_uint64(0)
        t0 = time.perf_counter()
        check(lib().bgx_dma_copy_d2h(addr, dev.data_ptr(), n, 0, ctypes.byref(tk)), "copy")
        check(lib().bgx_dma_wait(tk.value, 10000), "wait")
        ts.append((time.perf_counter() - t0) * 1e6)
    ok = bool(np.array_equal(np.frombuffer(shm.buf, np.int32)[: n // 4], np.arange(n // 4, dtype=np.int32)))
    med = float(np.median(ts))
    out[f"{mb}MiB"] = {"median_us": round(med, 1), "GBps": round(n / med / 1e3, 1), "content_ok": ok}
print(json.dumps(out))
lib().bgx_host_unregister(addr)
shm.close()
shm.unlink()
