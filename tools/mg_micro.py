#!/usr/bin/env python3
"""Movegen micro-benchmark: time bgx_movegen on self-play positions, split
into non-doubles and doubles jobs (tools only; positions come from the CPU
oracle's random play, results are not checked here — tests/ do that)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd"), os.path.join(REPO, "oracle")]
import oracle as orc  # noqa: E402  (input generation only)
from bgx import ops  # noqa: E402


def positions(seed, n_games):
    rng = np.random.default_rng(seed)
    init = np.array([2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 5, 0, 0, 0, 0, 3, 0, 5, 0, 0, 0, 0, 0,
                     0, 0, 0, 0, 0, 5, 0, 3, 0, 0, 0, 0, 5, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 0, 0, 0, 0], np.uint8)
    out = []
    for _ in range(n_games):
        b, pl = init.copy(), int(rng.integers(0, 2))
        for _s in range(300):
            out.append((b.copy(), pl))
            n, res, _ = orc.movegen(b, pl, int(rng.integers(1, 7)), int(rng.integers(1, 7)))
            if n:
                b = res[int(rng.integers(0, min(n, 500)))].copy()
                if b[50 + pl] >= 15:
                    break
            pl = 1 - pl
    return out


def time_it(boards, player, dice, cap, reps=20):
    b = torch.from_numpy(boards).cuda()
    p = torch.from_numpy(player).cuda()
    d = torch.from_numpy(dice).cuda()
    ops.movegen(b, p, d, cap=cap)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        out, cnt = ops.movegen(b, p, d, cap=cap)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    return ms, int(cnt.sum().item())


def main():
    pos = positions(7, 60)
    rng = np.random.default_rng(1)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    idx = rng.integers(0, len(pos), size=n)
    boards = np.stack([pos[i][0] for i in idx])
    player = np.array([pos[i][1] for i in idx], np.uint8)
    only = sys.argv[2] if len(sys.argv) > 2 else None
    res = {}
    for name, gen in (("nondoubles", lambda: (lambda a, b: np.where(a == b, (a % 6) + 1, b))(
                          rng.integers(1, 7, n), rng.integers(1, 7, n))),
                      ("doubles", None), ("mixed21", None)):
        if only and name != only:
            continue
        if name == "nondoubles":
            a = rng.integers(1, 7, n)
            b = rng.integers(1, 7, n)
            b = np.where(a == b, (a % 6) + 1, b)
            dice = np.stack([a, b], 1).astype(np.uint8)
        elif name == "doubles":
            a = rng.integers(1, 7, n)
            dice = np.stack([a, a], 1).astype(np.uint8)
        else:
            rolls = [(x, y) for x in range(1, 7) for y in range(x, 7)]
            r = rng.integers(0, 21, n)
            dice = np.array([rolls[k] for k in r], np.uint8)
        ms, tot = time_it(boards, player, dice, cap=4)
        res[name] = {"jobs": n, "ms": ms, "jobs_per_s": n / ms * 1e3, "results": tot, "us_per_job_wave": None}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
