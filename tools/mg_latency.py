#!/usr/bin/env python3
"""Movegen latency probe (tools only): launch time of a 1-ply-sized job set
(4096 self-play positions, random dice), the same with doubles swapped out,
only its doubles, and single heavy jobs (golden cases with the most results)."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mlp-ppo-2ply-multi_amd"), os.path.join(REPO, "tools"), os.path.join(REPO, "tests")]
from bgx import ops  # noqa: E402
from mg_micro import positions  # noqa: E402


def t_launch(boards, player, dice, reps=50):
    b = torch.from_numpy(np.ascontiguousarray(boards)).cuda()
    p = torch.from_numpy(np.ascontiguousarray(player)).cuda()
    d = torch.from_numpy(np.ascontiguousarray(dice)).cuda()
    ops.movegen(b, p, d, cap=4)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.movegen(b, p, d, cap=4)
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return float(np.median(ts)) * 1e3   # us


def main():
    pos = positions(7, 60)
    rng = np.random.default_rng(5)
    idx = rng.integers(0, len(pos), 4096)
    boards = np.stack([pos[i][0] for i in idx])
    player = np.array([pos[i][1] for i in idx], np.uint8)
    dice = rng.integers(1, 7, (4096, 2)).astype(np.uint8)
    dbl = dice[:, 0] == dice[:, 1]
    nd = dice.copy()
    nd[dbl, 1] = nd[dbl, 0] % 6 + 1
    res = {"mixed_4096": t_launch(boards, player, dice), "nondoubles_4096": t_launch(boards, player, nd),
           "doubles_only": t_launch(boards[dbl], player[dbl], dice[dbl]), "n_doubles": int(dbl.sum())}
    g = np.load(os.path.join(REPO, "tests", "golden", "movegen_cases.npz"))
    cnt = np.diff(g["offsets"])
    for k in np.argsort(-cnt)[:3]:
        res[f"single_{int(cnt[k])}_results"] = t_launch(g["boards"][k:k + 1], g["player"][k:k + 1], g["dice"][k:k + 1])
    res["single_empty_board_job"] = t_launch(g["boards"][:1], g["player"][:1], np.array([[3, 1]], np.uint8))
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
