"""Host emulation of the 2-ply reply launch against the oracle (tooling).

Builds tests/cpuwave/reply_emu.cpp with the given defines (default: the
shipped ones) and runs it on the positions of tests/test_gpu_reply.py
(self-play fuzz + random placements), EMU_N_CU emulated CUs (256 = the
GPU's grid), then checks every (board, roll) list against the oracle's
movegen, order included.

  python tools/emu_reply_check.py [--n-cu 256] [--roots N] [--runs R] [-D NAME=V ...] [--sites]
"""
import argparse
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "oracle"), os.path.join(REPO, "mlp-ppo-2ply-multi_amd")]

import oracle as orc  # noqa: E402
from test_cpuwave import _pack, _unpack  # noqa: E402
from test_gpu_parity import _fuzz_positions, _random_positions  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-cu", type=int, default=256)
    ap.add_argument("--roots", type=int, default=0, help="0 = all of test_gpu_reply's positions")
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--sites", action="store_true", help="EMU_SITES build (-O0 -fno-inline): uniformity only")
    ap.add_argument("--csrc", default=os.path.join(REPO, "mlp-ppo-2ply-multi_amd", "csrc"),
                    help="device sources to emulate (e.g. an older tree's csrc, from a git worktree)")
    a = ap.parse_args()
    pos = _fuzz_positions(77, 24) + _random_positions(5, 1500)
    if a.roots:
        pos = pos[:a.roots]
    boards = np.stack([p[0] for p in pos])
    opp = np.array([p[1] for p in pos], np.uint8)
    rows = np.zeros((len(pos), 9), np.uint32)
    rows[:, :8] = _pack(boards, 1 - opp.astype(np.uint32))
    rows[:, 8] = opp
    tmp = tempfile.mkdtemp(prefix="emu_reply_")
    pfile = os.path.join(tmp, "pos.bin")
    rows.tofile(pfile)
    exe = os.path.join(tmp, "reply_emu")
    opt = ["-O0", "-fno-inline", "-DEMU_SITES"] if a.sites else ["-O1", "-fsanitize=address", "-fno-omit-frame-pointer"]
    cmd = ["g++", "-std=c++20", *opt, "-g", "-w", *["-D" + d for d in a.D],
           "-I" + os.path.join(REPO, "tests", "cpuwave"), "-I" + a.csrc,
           "-I" + os.path.join(a.csrc, "..", "..", "include"), "-x", "c++",
           os.path.join(REPO, "tests", "cpuwave", "reply_emu.cpp"),
           "-o", exe, "-pthread"]
    subprocess.run(cmd, check=True)
    env = {**os.environ, "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=0", "EMU_N_CU": str(a.n_cu)}
    ref = {}
    rolls = [(x, y) for x in range(1, 7) for y in range(x, 7)]
    total_bad = 0
    for run in range(a.runs):
        dump = os.path.join(tmp, "dump.bin")
        t0 = time.time()
        r = subprocess.run([exe, pfile, str(len(pos)), dump], capture_output=True, text=True, env=env)
        print(f"run {run}: rc {r.returncode}, {time.time() - t0:.0f} s, {r.stdout.strip()}", flush=True)
        if r.returncode not in (0, 5):   # 5: some job left job_off / job_cnt unwritten (lists still compared)
            print(r.stderr[-3000:])
            sys.exit(1)
        total_bad += r.returncode == 5
        if a.sites:
            continue
        d = np.fromfile(dump, np.int32)
        at, bad = 0, []
        for i in range(len(pos)):
            for q, (x, y) in enumerate(rolls):
                c = int(d[at])
                at += 1
                got = _unpack(d[at:at + 8 * max(c, 0)].view(np.uint32).reshape(-1, 8)) if c > 0 else np.zeros((0, 52))
                at += 8 * max(c, 0)
                if (i, q) not in ref:
                    n, res, _ = orc.movegen(boards[i], int(opp[i]), x, y, cap=4096)
                    ref[(i, q)] = (n, res[:n].copy())
                n, res = ref[(i, q)]
                if c != n or not np.array_equal(got, res):
                    bad.append((i, x, y, c, n))
        assert at == d.shape[0]
        print(f"run {run}: {len(bad)} wrong lists of {len(pos) * 21}", bad[:10], flush=True)
        total_bad += len(bad)
    sys.exit(1 if total_bad else 0)


if __name__ == "__main__":
    main()
