"""Host-emulated wavefront checks of movegen device code (tests/cpuwave/).

The device headers are compiled for the host against tests/cpuwave/hip/
hip_runtime.h, which runs each of a wave's 64 lanes as a thread and every
cross-lane operation as an exchange between barriers; the build uses
AddressSanitizer, so a stray LDS-slice or output access aborts with a report.

test_board_major_doubles_equals_per_roll: the board-major doubles item
(board_dbl_emit, the six (d, d) rolls of a reply root expanded together,
bgx_movegen.h) gives every (root, die) the records of the per-roll path
(run_job: path_doubles_emit / job_records, which the GPU reply tests check
against the oracle), in the same order, written only inside the job's
reserved rows; the non-doubles item (board_nd_records2) runs first on the same
slice and must leave the parent map zero. Random positions (bar 0-2, borne-off
checkers). The 3,650 positions of tests/test_gpu_reply.py passed the same
check (tools: `dbl_check 4000 1 positions.bin`, ~9 min).
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_board_major_doubles_equals_per_roll(tmp_path):
    exe = tmp_path / "dbl_check"
    subprocess.run(["g++", "-std=c++20", "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-I" + os.path.join(HERE, "cpuwave"),
                    "-I" + os.path.join(REPO, "mlp-ppo-2ply-multi_amd", "csrc"),
                    "-I" + os.path.join(REPO, "include"),
                    os.path.join(HERE, "cpuwave", "dbl_check.cpp"), "-o", str(exe), "-pthread"],
                   check=True, capture_output=True, text=True)
    env = {**os.environ, "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=0"}
    r = subprocess.run([str(exe), "40", "7"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert '"mismatches": 0' in r.stdout, r.stdout[-2000:]
    assert '"board_major_roots": 0' not in r.stdout   # the board-major path actually ran
