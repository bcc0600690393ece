"""Which copy path moves a harvest-sized buffer device -> host on the DMA
engines (no kernel) while a kernel occupies every CU? Run under
  rocprofv3 --kernel-trace --memory-copy-trace -d DIR -o run --output-format csv -- python tools/copy_probe.py
Variants (each a 16 MiB device buffer, 4 copies, host-timed):
  shm_default / shm_d2h: into a shared-memory segment page-locked with
      bgx_host_register, bgx_copy_async kind 0 / 2
  pinned_d2h: into a torch pinned tensor (hipHostMalloc), bgx_copy_async kind 2
  torch_pinned: torch .copy_(non_blocking=True) into the same pinned tensor
  shm_nocu / pinned_nocu / d2d_nocu: hipMemcpyDeviceToDeviceNoCU (kind 4) into the
      registered segment / the pinned tensor / another device buffer
  shm_sdma: bgx_dma_copy_d2h (SDMA engine through HSA) into the registered segment
Development tool."""
import os
import sys
import time
from multiprocessing import shared_memory

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))
from bgx._lib import check, lib  # noqa: E402

N = 16 << 20
dev = torch.empty(N // 4, dtype=torch.int32, device="cuda").fill_(7)
shm = shared_memory.SharedMemory(create=True, size=N)
addr = np.frombuffer(shm.buf, np.uint8).ctypes.data
check(lib().bgx_host_register(addr, N), "register")
pinned = torch.empty(N // 4, dtype=torch.int32, pin_memory=True)
s = torch.cuda.Stream()
res = {}
dev2 = torch.empty_like(dev)
import ctypes  # noqa: E402
for name in ("shm_default", "shm_d2h", "pinned_d2h", "torch_pinned", "shm_nocu", "pinned_nocu", "d2d_nocu",
             "shm_sdma"):
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            if name == "shm_default":
                check(lib().bgx_copy_async(addr, dev.data_ptr(), N, 0, s.cuda_stream), name)
            elif name == "shm_d2h":
                check(lib().bgx_copy_async(addr, dev.data_ptr(), N, 2, s.cuda_stream), name)
            elif name == "pinned_d2h":
                check(lib().bgx_copy_async(pinned.data_ptr(), dev.data_ptr(), N, 2, s.cuda_stream), name)
            elif name == "shm_nocu":
                check(lib().bgx_copy_async(addr, dev.data_ptr(), N, 4, s.cuda_stream), name)
            elif name == "pinned_nocu":
                check(lib().bgx_copy_async(pinned.data_ptr(), dev.data_ptr(), N, 4, s.cuda_stream), name)
            elif name == "shm_sdma":
                tk = ctypes.c_uint64(0)
                check(lib().bgx_dma_copy_d2h(addr, dev.data_ptr(), N, 0, ctypes.byref(tk)), name)
                check(lib().bgx_dma_wait(tk.value, 10000), name)
            elif name == "d2d_nocu":
                check(lib().bgx_copy_async(dev2.data_ptr(), dev.data_ptr(), N, 4, s.cuda_stream), name)
            else:
                pinned.copy_(dev, non_blocking=True)
        s.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    res[name] = round(float(np.median(ts)), 1)
    torch.cuda.synchronize()
    time.sleep(0.01)
print({k: f"{v} us ({N / v / 1e3:.1f} GB/s)" for k, v in res.items()})
assert np.frombuffer(shm.buf, np.int32)[123] == 7
assert int(pinned[123]) == 7
lib().bgx_host_unregister(addr)
shm.close()
shm.unlink()
