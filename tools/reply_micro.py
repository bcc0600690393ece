#!/usr/bin/env python3
"""2-ply reply-launch micro-benchmark (tools only): the reply movegen over N
candidate boards from the CPU oracle's random self-play (inputs only; tests/
check the results), timed per kernel with HIP events, for the board-major
kernel (default), the per-roll kernel (BGX_REPLY_BM=0) and, with
BGX_REPLY_GROUPS, one item group at a time (0x1: the 15 non-doubles rolls,
0x7e: the six doubles). One JSON line."""
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]


def run_one(n, reps):
    import torch
    from bgx import ops
    from test_gpu_parity import _fuzz_positions
    pos = _fuzz_positions(3, max(1, n // 150))
    rng = np.random.default_rng(0)
    idx = rng.integers(0, len(pos), n)
    boards = torch.from_numpy(np.stack([pos[i][0] for i in idx])).cuda()
    opp = torch.from_numpy(np.array([pos[i][1] for i in idx], np.uint8)).cuda()
    cap = n * 21 * 64 + 4096
    ops.reply_moves(boards, opp, cap=cap)
    torch.cuda.synchronize()
    import time
    t0 = time.perf_counter()
    for _ in range(reps):
        _, _, cnt = ops.reply_moves(boards, opp, cap=cap)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
    if len(sys.argv) > 2 and sys.argv[2] == "child":
        print(json.dumps({"ms_per_call": run_one(n, 10)}))
        return
    out = {"boards": n}
    for name, env in (("board_major", {}), ("per_roll", {"BGX_REPLY_BM": "0"}),
                      ("bm_nondoubles_only", {"BGX_REPLY_GROUPS": "0x1"}),
                      ("bm_doubles_only", {"BGX_REPLY_GROUPS": "0x7e"})):
        r = subprocess.run([sys.executable, __file__, str(n), "child"], env={**os.environ, **env,
                           "BGX_MG_FEW": "0"}, capture_output=True, text=True, check=True)
        out[name] = json.loads(r.stdout.strip().splitlines()[-1])["ms_per_call"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
