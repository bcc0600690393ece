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

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CLANG = "/opt/rocm/lib/llvm/bin/clang++"


def _emu_sources(tmp_path):
    """A copy of csrc/ for host builds: the inline-asm scheduling hints
    (`asm volatile(...)`: waitcnts, register pins) removed and each dynamic LDS
    array (`extern __shared__ T x[];`) bound to the emulated workgroup's buffer.
    The kernels' code is otherwise the product's, unchanged."""
    import glob
    import re
    d = tmp_path / "csrc_emu"
    d.mkdir(exist_ok=True)
    for f in glob.glob(os.path.join(REPO, "mlp-ppo-2ply-multi_amd", "csrc", "*.h")) + \
            glob.glob(os.path.join(REPO, "mlp-ppo-2ply-multi_amd", "csrc", "*.hip")):
        s = open(f).read()
        s = re.sub(r"asm volatile\((?:[^;])*?\);", ";", s)
        s = re.sub(r"extern __shared__ (?:__attribute__\(\(aligned\(\d+\)\)\) )?([\w ]+?) (\w+)\[\];",
                   r"\1* \2 = (\1*)emu::dyn_lds;", s)
        (d / os.path.basename(f)).write_text(s)
    return d


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


def _build(tmp_path, src, name, defs=()):
    exe = tmp_path / name
    subprocess.run(["g++", "-std=c++20", "-O1", "-g", "-w", "-fsanitize=address", "-fno-omit-frame-pointer",
                    *defs, "-I" + os.path.join(HERE, "cpuwave"),
                    "-I" + os.path.join(REPO, "mlp-ppo-2ply-multi_amd", "csrc"),
                    "-I" + os.path.join(REPO, "include"), "-x", "c++",
                    os.path.join(HERE, "cpuwave", src), "-o", str(exe), "-pthread"],
                   check=True, capture_output=True, text=True)
    return exe


def _unpack(w):
    """packed rows uint32 [n, 8] -> uint8 [n, 52] (bgx_device.h packed_to_u8)"""
    n = w.shape[0]
    out = np.zeros((n, 52), np.uint8)
    for k in range(6):
        for q in range(8):
            out[:, 8 * k + q] = (w[:, k] >> (4 * q)) & 15
    for i in range(4):
        out[:, 48 + i] = (w[:, 6] >> (4 * i)) & 15
    return out


def _reply_vs_oracle(tmp_path, defs, n_cu=2):
    """The reply launch emulated (per-roll doubles items and the board-major
    doubles kernel, BGX_REPLY_DBL=0 / 1, the latter with half its rows in
    per-roll items, BGX_REPLY_DBL_TAIL=32; extra defs) on self-play and random
    positions over n_cu emulated CUs: both kernels' per-job output
    byte-identical, and every (board, roll) list the oracle's, order included."""
    orc = pytest.importorskip("oracle")
    from test_gpu_parity import _fuzz_positions, _random_positions
    pos = _fuzz_positions(11, 4) + _random_positions(12, 90)
    boards = np.stack([p[0] for p in pos])
    opp = np.array([p[1] for p in pos], np.uint8)
    rows = np.zeros((len(pos), 9), np.uint32)
    rows[:, :8] = _pack(boards, 1 - opp.astype(np.uint32))
    rows[:, 8] = opp
    pfile = tmp_path / "pos.bin"
    rows.tofile(pfile)
    dumps = []
    exe = _build(tmp_path, "reply_emu.cpp", "reply_emu", list(defs))
    for v in ("0", "1"):
        env = {**os.environ, "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=0", "EMU_N_CU": str(n_cu),
               "BGX_REPLY_DBL": v, "BGX_REPLY_DBL_TAIL": "32"}
        dump = tmp_path / ("dump" + v + ".bin")
        r = subprocess.run([str(exe), str(pfile), str(len(pos)), str(dump)], capture_output=True, text=True,
                           timeout=900, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        dumps.append(dump.read_bytes())
    assert dumps[0] == dumps[1]
    d = np.frombuffer(dumps[0], np.int32)
    at = 0
    rolls = [(a, b) for a in range(1, 7) for b in range(a, 7)]
    for i in range(len(pos)):
        for a, b in rolls:
            c = int(d[at])
            at += 1
            got = _unpack(d[at:at + 8 * max(c, 0)].view(np.uint32).reshape(-1, 8)) if c > 0 else np.zeros((0, 52))
            at += 8 * max(c, 0)
            n, res, _ = orc.movegen(boards[i], int(opp[i]), a, b, cap=4096)
            assert c == n, (i, a, b, c, n)
            np.testing.assert_array_equal(got, res[:n], err_msg=f"board {i} roll {a}-{b}")
    assert at == d.shape[0]


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_reply_launch_emulated_equals_oracle(tmp_path):
    """The whole 2-ply reply launch as bgx_reply_moves issues it (reply kernel:
    16-wave workgroups, per-roll calls; then the tier-2 block kernel), emulated
    on the host under AddressSanitizer: every (board, roll) list equals the
    oracle's movegen (generate_all_moves.py:7-90), order included, with the
    per-roll doubles items and with the board-major doubles kernel
    (BGX_REPLY_DBL=1, the K = all launch's), whose per-job output is
    byte-identical. Built with the
    workgroup sub-queue off (BGX_REPLY_SUBQ=0: an uncovered root's 15 per-roll
    jobs run on its own wave); the sub-queue is the next test's."""
    _reply_vs_oracle(tmp_path, ["-DBGX_REPLY_SUBQ=0"])


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_reply_launch_emulated_with_subqueue_equals_oracle(tmp_path):
    """As above with the sub-queue that shares an uncovered root's 15 per-roll
    jobs among the workgroup's waves (the shipped configuration), over 64
    emulated CUs: most waves of a workgroup draw no item and sit in the exit
    test while the others push sub-jobs -- the timing under which a per-lane
    exit test once split waves (round 4: 11-27 wrong late-row lists per 76,650
    at 256 CUs; the exit verdict is now lane 0's, broadcast)."""
    _reply_vs_oracle(tmp_path, [], n_cu=64)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_reply_launch_cross_lane_ops_are_uniform(tmp_path):
    """Every cross-lane operation of the reply launch (ballot, shuffles,
    readlane, DPP scans) is reached by all 64 lanes of the wave from the same
    call chain (EMU_SITES build, -O0 -fno-inline): on the GPU one under
    lane-divergent control flow would read inactive lanes. Both builds
    (per-roll and board-major doubles, half its rows per roll), with the
    shipped sub-queue, over 16
    emulated CUs (waves that draw no item sit in the exit test); the emulation
    itself aborts on a kernel that branches around a shuffle (checked with a
    deliberately divergent one). (Round 4's per-lane exit test once left lanes
    of a wave at two different call sites here; its verdict is now lane 0's,
    broadcast.)"""
    from test_gpu_parity import _random_positions
    pytest.importorskip("oracle")
    pos = _random_positions(21, 40)
    boards = np.stack([p[0] for p in pos])
    opp = np.array([p[1] for p in pos], np.uint8)
    rows = np.zeros((len(pos), 9), np.uint32)
    for k in range(6):
        for q in range(8):
            rows[:, k] |= boards[:, 8 * k + q].astype(np.uint32) << np.uint32(4 * q)
    rows[:, 6] = (boards[:, 48].astype(np.uint32) | boards[:, 49].astype(np.uint32) << 4 |
                  boards[:, 50].astype(np.uint32) << 8 | boards[:, 51].astype(np.uint32) << 12 |
                  (1 - opp.astype(np.uint32)) << 16)
    rows[:, 8] = opp
    pfile = tmp_path / "pos.bin"
    rows.tofile(pfile)
    inc = ["-I" + os.path.join(HERE, "cpuwave"), "-I" + os.path.join(REPO, "mlp-ppo-2ply-multi_amd", "csrc"),
           "-I" + os.path.join(REPO, "include")]
    bad = tmp_path / "bad.cpp"
    bad.write_text('#include "hip/hip_runtime.h"\n'
                   "__global__ void k(int* o) { int v = (int)threadIdx.x; int r;\n"
                   "  if (threadIdx.x & 1) r = __shfl(v, 0, 64); else r = __shfl(v, 1, 64); o[threadIdx.x] = r; }\n"
                   "int main() { static int o[64]; hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, nullptr, o); }\n")
    exe = tmp_path / "bad"
    subprocess.run(["g++", "-std=c++20", "-O0", "-fno-inline", "-g", "-w", "-DEMU_SITES", *inc, "-x", "c++", str(bad),
                    "-o", str(exe), "-pthread"], check=True, capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "EMU_SITES" in r.stderr
    exe = tmp_path / "site"
    subprocess.run(["g++", "-std=c++20", "-O0", "-fno-inline", "-g", "-w", "-DEMU_SITES", *inc, "-x", "c++",
                    os.path.join(HERE, "cpuwave", "reply_emu.cpp"), "-o", str(exe), "-pthread"], check=True,
                   capture_output=True, text=True)
    for v in ("0", "1"):
        r = subprocess.run([str(exe), str(pfile), str(len(pos)), str(tmp_path / ("s" + v))], capture_output=True,
                           text=True, timeout=900, env={**os.environ, "EMU_N_CU": "16", "BGX_REPLY_DBL": v,
                                                        "BGX_REPLY_DBL_TAIL": "32"})
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]


def _pack(boards, flag):
    rows = np.zeros((len(boards), 8), np.uint32)
    for k in range(6):
        for q in range(8):
            rows[:, k] |= boards[:, 8 * k + q].astype(np.uint32) << np.uint32(4 * q)
    rows[:, 6] = (boards[:, 48].astype(np.uint32) | boards[:, 49].astype(np.uint32) << 4 |
                  boards[:, 50].astype(np.uint32) << 8 | boards[:, 51].astype(np.uint32) << 12 |
                  np.asarray(flag).astype(np.uint32) << 16)
    return rows


@pytest.mark.skipif(not os.path.exists(CLANG), reason="no ROCm clang")
def test_mlp_kernels_emulated_equal_oracle_value(tmp_path):
    """The MLP launch (bgx_launch_mlp: the 16-wave single-tile kernel and the
    8-wave interleaved-epilogue kernel), emulated on the host with the
    v_mfma_f32_32x32x16_f16 operand layout, gives the oracle's fp64 value
    (policy_network.py:53-70) within 1e-6 on the shipped checkpoint for random
    placements (bar, borne-off checkers): the fragment layout (bgx_frag.h), the
    LUT features, the split-fp16 product and the epilogue, checked without a
    GPU. AddressSanitizer on."""
    orc = pytest.importorskip("oracle")
    from test_gpu_parity import _random_positions
    pos = _random_positions(3, 150)
    boards = np.stack([p[0] for p in pos])
    pl = np.array([p[1] for p in pos])
    _pack(boards, pl).tofile(tmp_path / "rows.bin")
    w = np.load(os.path.join(HERE, "golden", "weights_ckpt2100000.npz"))
    W = {k: w[k].astype(np.float32) for k in ("W1", "b1", "w2", "b2")}
    np.concatenate([W[k].ravel() for k in ("W1", "b1", "w2", "b2")]).astype(np.float32).tofile(tmp_path / "w.bin")
    ref = orc.value(W, orc.encode_many(boards, pl))
    src = _emu_sources(tmp_path)
    exe = tmp_path / "mlp_emu"
    subprocess.run([CLANG, "-std=c++20", "-O1", "-g", "-w", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-I" + str(src), "-I" + os.path.join(HERE, "cpuwave"), "-I" + os.path.join(REPO, "include"),
                    "-x", "c++", os.path.join(HERE, "cpuwave", "mlp_emu.cpp"), "-o", str(exe), "-pthread"],
                   check=True, capture_output=True, text=True)
    env = {**os.environ, "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=0"}
    for nt in ("1", "2"):
        out = tmp_path / ("v" + nt + ".bin")
        r = subprocess.run([str(exe), str(tmp_path / "rows.bin"), str(tmp_path / "w.bin"), nt, str(out)],
                           capture_output=True, text=True, timeout=600, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        v = np.fromfile(out, np.float32)
        assert v.shape == ref.shape
        assert np.abs(v - ref).max() < 1e-6, (nt, np.abs(v - ref).max())


@pytest.mark.skipif(not os.path.exists(CLANG), reason="no ROCm clang")
def test_mlp_delta_kernel_emulated_equals_oracle_value(tmp_path):
    """The 2-ply reply MLP by difference from the root (mlp_kernel_delta: the
    root launch writes its hidden accumulators, each reply row -- word 7 = its
    root -- adds W . (x_reply - x_root) over the tile's changed byte groups),
    emulated on the host: the replies to 40 random positions for all 21 rolls
    (tens of thousands of rows, tiles spanning several roots) give the oracle's
    fp64 value (policy_network.py:53-70) within 2e-6 on the shipped checkpoint.
    AddressSanitizer on (the root / accumulator gathers stay in bounds, also for
    a stale root index, which is clamped)."""
    orc = pytest.importorskip("oracle")
    from test_gpu_parity import _random_positions
    pos = _random_positions(8, 40)
    rolls = [(a, b) for a in range(1, 7) for b in range(a, 7)]
    roots, reps, slot, opp = [], [], [], []
    for i, (board, mover) in enumerate(pos):
        o = 1 - int(mover)   # the replier; the root's indicator is the player who moved
        roots.append(_pack(board[None], np.array([mover]))[0])
        for a, b in rolls:
            n, res, _ = orc.movegen(board, o, a, b)
            reps += list(res[:n])
            slot += [i] * n
            opp += [o] * n
    reps = np.stack(reps)
    rows = _pack(reps, np.array(opp))
    rows[:, 7] = np.array(slot, np.uint32)
    rows[-1, 7] = 0xFFFFFFF0   # a stale root index: clamped (its V is still computed, from some root)
    rows.tofile(tmp_path / "rows.bin")
    np.stack(roots).astype(np.uint32).tofile(tmp_path / "roots.bin")
    w = np.load(os.path.join(HERE, "golden", "weights_ckpt2100000.npz"))
    W = {k: w[k].astype(np.float32) for k in ("W1", "b1", "w2", "b2")}
    np.concatenate([W[k].ravel() for k in ("W1", "b1", "w2", "b2")]).astype(np.float32).tofile(tmp_path / "w.bin")
    ref = orc.value(W, orc.encode_many(reps, opp))
    src = _emu_sources(tmp_path)
    exe = tmp_path / "mlp_emu"
    subprocess.run([CLANG, "-std=c++20", "-O1", "-g", "-w", "-fsanitize=address", "-fno-omit-frame-pointer",
                    "-I" + str(src), "-I" + os.path.join(HERE, "cpuwave"), "-I" + os.path.join(REPO, "include"),
                    "-x", "c++", os.path.join(HERE, "cpuwave", "mlp_emu.cpp"), "-o", str(exe), "-pthread"],
                   check=True, capture_output=True, text=True)
    env = {**os.environ, "ASAN_OPTIONS": "verify_asan_link_order=0:detect_leaks=0"}
    out = tmp_path / "vd.bin"
    r = subprocess.run([str(exe), str(tmp_path / "rows.bin"), str(tmp_path / "w.bin"), "d", str(out),
                        str(tmp_path / "roots.bin")], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    v = np.fromfile(out, np.float32)
    assert v.shape == ref.shape and len(v) > 10000
    err = np.abs(v[:-1] - ref[:-1])
    assert err.max() < 2e-6, (err.max(), int(err.argmax()))
