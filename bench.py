#!/usr/bin/env python3
"""Self-play throughput benchmark (BASELINE.json metric: self-play env steps/sec).

One bench "step" = one env step (one BackgammonEnv.step equivalent, passes
included) of every lane on every GPU, including the compact Experience
records, the episode harvest (every --harvest-every steps) and, for N > 1,
the RCCL gather of the harvested episodes to rank 0. Synthetic data: lanes
start from the reference's reset and play random-seeded self-play with the
seeded xavier weights (tests/golden/weights_seed0.npz = torch.manual_seed(0)
BackgammonPolicyNetwork()), T = 1.5 (ParameterManager version 1).

Workload: 8,192 game lanes per GPU (weak scaling; N = 8 is configs[3]/[4]'s
65,536 lanes sharded across 8 MI355X), 1-ply softmax select as the headline,
with 2-ply K=4 (configs[4]) and K=all (configs[2]'s ~21 x C reply boards per
decision) legs on the same lanes, and at N = 1 configs[1] (4,096 lanes) beside.

N = 1:  python bench.py
N > 1:  python bench.py --gpus N      (starts N rank processes itself through
            torch.distributed.run before anything touches a GPU), or as the
            driver does: python -m torch.distributed.run --nnodes=1
            --nproc-per-node N --master-addr 127.0.0.1 --master-port P
            bench.py --gpus N
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mlp-ppo-2ply-multi_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP16_DENSE_PEAK_TFS = 2500.0  # dense fp16 MFMA (no sparsity)
MLP_FLOP_PER_ROW = 50944     # 2 * (198*128 + 128)  
MOVEGEN_BYTES_PER_JOB = 54   # parent board + player + dice
MOVEGEN_BYTES_PER_ROW = 52   # child board written
PIPELINE_BYTES_PER_BOARD = 901   # canonical unfused pipeline per evaluated board: child write 52
                                 # + encode read 53 + fp16 feature write 396 + MLP read 396 + V write 4
METRIC = "self-play env steps/sec (whole node) at 1-ply and 2-ply, 1/2/4/8 MI355X"


def load_weights():
    d = np.load(os.path.join(REPO, "tests", "golden", "weights_seed0.npz"))
    return {k: d[k] for k in ("W1", "b1", "w2", "b2")}


BACKEND = os.environ.get("BGX_DIST_BACKEND", "nccl")   # "gloo": rehearsal with ranks sharing GPUs
FAIL_RANK = int(os.environ.get("BGX_BENCH_FAIL_RANK", "-1"))   # test hook: this rank raises mid-run


def _coll_device():
    return torch.device("cuda", torch.cuda.current_device()) if BACKEND == "nccl" else torch.device("cpu")


def init_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(BACKEND)
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_ranks(x, world):
    """x from every rank, in rank order."""
    if world == 1:
        return [x]
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device())
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(o.item()) for o in out]


def sum_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def run_engine(args, world, rank, ply, k_top, lanes, steps, warmup, harvest_every, timing, timing_steps=0,
               desync=0, seed=None):
    from bgx import Engine
    from bgx import dist as bdist
    w = load_weights()
    if world > 1:
        w = bdist.broadcast_weights(w)
    eng = Engine(lanes=lanes, seed=args.seed if seed is None else seed, ply=ply, k_top=k_top, lane_base=rank * lanes,
                 fused=not args.no_fused, balance=not args.no_balance)
    eng.set_weights(w, temperature=1.5, version=1)
    gathered = [0, 0]
    harvested = [0, 0]   # this rank's own harvests (episodes, records), every run() of the engine
    collect_t = [0.0, 0]   # rank 0: seconds inside hg.collect (+ its copies at --collect-copy), batches
    hg = None
    if world > 1 and args.gather in ("host", "device"):
        from bgx import devgather, hostgather
        # host: anonymous memory segments (memfd), not /dev/shm files, so the path
        # does not depend on the container's /dev/shm size (bgx/hostgather.py);
        # device: slots in rank 0's GPU memory, peer copies on the DMA engines
        # (bgx/devgather.py). Same protocol, no collective per harvest.
        mod = hostgather if args.gather == "host" else devgather
        hg = mod.setup(rank, world, hostgather.slot_bytes_for(lanes, args.harvest_every), dst=0,
                       device=torch.cuda.current_device())
    seq = [0]

    def run(n):
        # The harvest is queued behind each launch (harvest_enqueue) and the next
        # launch is queued before the host looks at it, so the device never waits
        # for the host; chunk i's episodes are handed on (gathered at N > 1) while
        # chunk i + 1 runs, and that hand-off is complete before the harvest
        # buffers it reads are reused (two harvests later).
        left, pending_t, inflight = n, None, None

        def consume(t):
            nonlocal inflight
            # the previous hand-off first: the loop's last consume and the final one
            # come back to back, and a Pending replaced without its wait() would
            # never publish its batch (rank 0 would read that slot's stale counts)
            settle()
            if world == 1:
                eng.harvest_fetch(t, wrap=False)   # the harvest ran on the device; nobody reads it here
                return
            h = eng.harvest_fetch(t)
            harvested[0] += h.n_episodes
            harvested[1] += h.n_records
            if FAIL_RANK == rank and seq[0] >= 1:   # test hook: this rank dies mid-run (after one batch)
                raise RuntimeError(f"BGX_BENCH_FAIL_RANK: rank {rank} fails on purpose")
            if hg is not None:      # DMA engines into host shared memory / rank 0's GPU; no collective
                seq[0] += 1
                if rank == 0:
                    tc = time.perf_counter()
                    # --collect-copy: the peers' batches cloned on rank 0's stream, as a GPU
                    # trainer takes them (devgather.collect synchronises that stream, which
                    # carries this rank's own persistent launch, before acknowledging)
                    parts = hg.collect(seq[0], copy=args.collect_copy)
                    collect_t[0] += time.perf_counter() - tc
                    collect_t[1] += 1
                    for part in parts:
                        if part is not None:
                            gathered[0] += part[0].shape[0]
                            gathered[1] += part[1].shape[0]
                    gathered[0] += h.n_episodes
                    gathered[1] += h.n_records
                    hg.ack(seq[0])
                else:
                    inflight = hg.publish(h, ready=True)   # harvest_fetch waited for the arrays
            else:                   # RCCL point-to-point to rank 0
                inflight = bdist.gather_episodes(h, dst=0, async_op=True)

        def settle():
            nonlocal inflight
            if inflight is not None:
                r = inflight.wait()
                if hg is None and rank == 0:
                    gathered[0] += r[0]
                    gathered[1] += r[1]
                inflight = None

        while left > 0:
            k = min(harvest_every, left)
            settle()               # the previous hand-off, before its buffers can be reused
            eng.step(k)
            t = eng.harvest_enqueue()
            if pending_t is not None:
                consume(pending_t)
            pending_t = t
            left -= k
        if pending_t is not None:
            consume(pending_t)
        settle()

    # lanes start together from the reset; `desync` untimed steps
    # (harvested, and gathered at N > 1, like the timed ones) spread them over
    # their games so the timed window holds finished episodes, refills and
    # harvests, then the driver's warmup. The desync lasts at least
    # --desync-ms of GPU time too (more chunks of --harvest-every steps): 300
    # 1-ply steps are ~11 ms, after which the driver's 20-step window still ran
    # ~4 % slower than after ~45 ms (220-225 vs 232-233 M env steps/s,
    # tools/runs/r6_desync.sh; the GPU idles during the CPU baseline before it)
    t_ds = time.perf_counter()
    run(desync)
    desync_run = desync
    while True:   # the same number of extra chunks on every rank (the gathers count batches)
        eng.sync()
        more = (time.perf_counter() - t_ds) * 1e3 < args.desync_ms
        if world > 1:
            more = max_over_ranks(1.0 if more else 0.0, world) > 0
        if not more:
            break
        run(harvest_every)
        desync_run += harvest_every
    run(warmup)
    eng.sync()
    s0 = eng.stats()
    c0 = list(collect_t)
    barrier(world)
    t0 = time.perf_counter()
    run(steps)          # direct launches, no events in the stream
    barrier(world)
    el = time.perf_counter() - t0
    s1 = eng.stats()
    d = {k: s1[k] - s0[k] for k in s1}
    d["collect_s"], d["collect_batches"] = collect_t[0] - c0[0], collect_t[1] - c0[1]   # the timed window's
    tm = d_tm = None
    if timing:
        # per-kernel durations: a second pass of the same workload with HIP
        # events recorded around every movegen / MLP launch on the engine stream
        eng.set_timing(True)
        t1 = time.perf_counter()
        run(timing_steps)
        eng.sync()
        el_tm = time.perf_counter() - t1
        s2 = eng.stats()
        tm = eng.timing()
        d_tm = {k: s2[k] - s1[k] for k in s2}
        d_tm["elapsed_s"] = el_tm
        d_tm["lanes"] = lanes
    eng.close()
    if hg is not None:
        import torch.distributed as dist
        dist.barrier()
        hg.close()
    d["desync_steps_run"] = desync_run
    return el, d, tm, d_tm, gathered, harvested


CPU_WARMUP_STEPS = 300   # BASELINE.md's CPU plan: a 300-step warm-up, then the timed window


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_worker(core, tasks, results):
    """One pinned CPU-baseline process: runs the tasks it is sent, in order."""
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        os.sched_setaffinity(0, {core})   # one host core per process (main.py:86's 7 workers)
    except (OSError, AttributeError):
        pass
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # the bench's cpu_baseline leg (oracle = the CPU port)
    w = load_weights()
    while True:
        t = tasks.get()
        if t is None:
            return
        seed, ply, seconds, warmup = t
        results.put(orc.selfplay_bench(w, temperature=1.5, seed=seed, n_threads=1, seconds=seconds, ply=ply,
                                       warmup=warmup))


def cpu_baseline(procs, seconds_1ply, seeds, seconds_2ply):
    """The CPU port of the worker loop (oracle/bgref.c, pinned by the golden
    fixtures) as `procs` processes, each pinned to its own host core: one
    1-ply round per seed, each process timing its window after a 300-step
    warm-up of whole games (BASELINE.md's plan; median of the per-round
    aggregates), then one 2-ply K=4 round whose 300-step warm-up plays 1-ply
    decisions (2-ply ones take ~30 ms each on a core) and ends mid-game, so
    the 2-ply window starts from the self-play position mix, not the
    openings. Runs before this process touches the GPU."""
    import multiprocessing as mp
    cores = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count()))
    ctx = mp.get_context("spawn")
    results = ctx.Queue()
    tasks = [ctx.Queue() for _ in range(procs)]
    ws = [ctx.Process(target=_cpu_worker, args=(cores[i % len(cores)], tasks[i], results), daemon=True)
          for i in range(procs)]
    for w in ws:
        w.start()

    def round_(seed, ply, seconds, warmup=0):
        for i in range(procs):
            tasks[i].put((1000 * seed + i, ply, seconds, warmup))
        rs = [results.get(timeout=600) for _ in range(procs)]
        return rs, max(r["elapsed"] for r in rs)

    out = {}
    try:
        rates = []
        for s in seeds:
            rs, el = round_(s, 1, seconds_1ply, warmup=CPU_WARMUP_STEPS)
            rates.append(sum(r["steps"] for r in rs) / el)
        out["1ply"] = {"rates": rates, "median": float(np.median(rates))}
        if seconds_2ply > 0:
            rs, el = round_(77, 2, seconds_2ply, warmup=CPU_WARMUP_STEPS)
            out["2ply"] = {"value": sum(r["steps"] for r in rs) / el,
                           "decisions_per_s": sum(r["decisions"] for r in rs) / el, "elapsed": el}
    finally:
        for q in tasks:
            q.put(None)
        for w in ws:
            w.join(timeout=60)
    out["cores_used"] = min(procs, len(cores))
    out["nproc"] = os.cpu_count()
    out["affinity"] = len(cores)
    out["cpu_model"] = _cpu_model()
    return out


def _pmc(leg, group, key, lanes=8192):
    """A per-launch PMC figure from the committed round profile
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py from separate
    rocprofv3 --pmc passes of this same bench workload), with its source.
    The profile's legs run at 8,192 lanes; a leg at another lane count reads
    its own l<lanes>_ entry or nothing (never the 8,192-lane figure)."""
    prof = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if lanes != 8192:
        leg = f"l{lanes}_{leg}"
    try:
        with open(prof) as f:
            j = json.load(f)
        v = j.get(leg, {}).get(group, {}).get(key)
        if v is None:
            return None, None
        src = f"profiles/pmc_traffic.json [{leg}] ({j.get('round', '?')}: {j.get('workload', '?')})"
        return v, src
    except (OSError, ValueError):
        return None, None


def roofline_fused(d, tm, lanes=8192):
    """The fused 1-ply step kernel (one launch = all steps of a step() call):
    the whole path's algorithmic bytes (54 B per movegen job +
    901 B per evaluated board) and MLP FLOPs over its average launch.

    The kernel is not HBM-bound: fusion keeps features and V on chip, so its
    physical traffic (PMC) is ~1/28 of the algorithmic bytes. Each step is one
    LDS item queue (MLP tiles on MFMA, choice chains, the next step's movegen
    jobs on VALU + SALU) that the waves of a workgroup share: the bound is
    issue and dependency latency across those items, not a single unit.
    `bound` says so; achieved / peak / frac stay the algorithmic-bytes figure
    of the bench contract, with the physical rate and the busy ratios beside it."""
    el = d["elapsed_s"]
    n = max(1, tm["movegen_launches"])
    launch = tm["movegen_ms"] / n
    byts = (MOVEGEN_BYTES_PER_JOB * d["movegen_jobs"] + PIPELINE_BYTES_PER_BOARD * d["value_rows"]) / n
    flop = MLP_FLOP_PER_ROW * d["value_rows"] / n
    k = {"bound": "hbm", "achieved": byts / (launch * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "avg_launch_ms": launch, "launches": n, "steps_per_launch": d["env_steps"] / max(1, d["lanes"]) / n,
         "share_of_wall": tm["movegen_ms"] * 1e-3 / el,
         "basis": "54 B per movegen job + 901 B per evaluated board (SURVEY 8d canonical pipeline)"}
    k["frac"] = k["achieved"] / k["peak"]
    m = {"bound": "mfma", "achieved": flop / (launch * 1e-3) / 1e12, "peak": FP16_DENSE_PEAK_TFS,
         "unit": "TFLOP/s", "avg_launch_ms": launch, "launches": n,
         "basis": "50,944 FLOP per evaluated board (fp16x2 split: 2x that on the MFMA pipes)"}
    m["frac"] = m["achieved"] / m["peak"]
    r = {kk: k[kk] for kk in ("achieved", "peak", "unit", "frac")}
    r["bound"] = "latency"
    r["bound_detail"] = ("VALU/SALU issue of the movegen items and dependency latency of the choice items, "
                         "sharing the SIMDs with the MLP tiles in one queue per step (not HBM: physical traffic "
                         "below; not MFMA: mfma_busy below)")
    r["kernel"] = "bgx::fused_step_kernel (movegen + encode + MLP + select + env step, all steps of a launch)"
    r["achieved_basis"] = "SURVEY 8d algorithmic bytes (54 B per movegen job + 901 B per evaluated board)"
    # PMC bytes per step of the same workload x the steps of this bench's launches
    per_step, src = _pmc("1ply_fused", "fused", "hbm_bytes_per_step", lanes)
    r["traffic"] = per_step * k["steps_per_launch"] if per_step else None
    r["traffic_source"] = src if per_step else None
    r["physical_gbs"] = r["traffic"] / (launch * 1e-3) / 1e9 if r["traffic"] else None
    r["physical_frac"] = r["physical_gbs"] / HBM_PEAK_GBS if r["physical_gbs"] else None
    for key in ("valu_busy", "mfma_busy", "lds_busy", "salu_busy", "wait_frac", "issue_stall_frac", "waves_per_cu"):
        r[key] = _pmc("1ply_fused", "fused", key, lanes)[0]
    r["mfma_frac_algorithmic"] = m["frac"]
    return r, {"fused_step": k, "fused_step_mfma": m}


def roofline_for(d, tm, leg, lanes=8192):
    """Dominant kernel's algorithmic rate over its average launch (HIP events),
    from the timed pass `d` (stats deltas) / `tm` (event totals)."""
    if tm["mlp_launches"] == 0 and tm["movegen_launches"] > 0:
        return roofline_fused(d, tm, lanes)
    el = d["elapsed_s"]
    mg_ms, mlp_ms = tm["movegen_ms"], tm["mlp_ms"]
    out = {}
    # boards movegen wrote = value rows minus the lanes' own rows (one per lane
    # step) and the reply launch's unwritten gap rows
    rec_rows = d["value_rows"] - d.get("gap_rows", 0)
    mg_rows = rec_rows - d["env_steps"]
    mg_bytes = MOVEGEN_BYTES_PER_JOB * d["movegen_jobs"] + MOVEGEN_BYTES_PER_ROW * mg_rows
    mg_launch = mg_ms / max(1, tm["movegen_launches"])
    out["movegen"] = {"bound": "hbm", "achieved": mg_bytes / max(1, tm["movegen_launches"]) / (mg_launch * 1e-3) / 1e9,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "avg_launch_ms": mg_launch,
                      "launches": tm["movegen_launches"], "share_of_wall": mg_ms * 1e-3 / el}
    mlp_launch = mlp_ms / max(1, tm["mlp_launches"])
    mlp_flop = MLP_FLOP_PER_ROW * rec_rows / max(1, tm["mlp_launches"])   # gap rows: executed, not counted
    out["mlp"] = {"bound": "mfma", "achieved": mlp_flop / (mlp_launch * 1e-3) / 1e12, "peak": FP16_DENSE_PEAK_TFS,
                  "unit": "TFLOP/s", "avg_launch_ms": mlp_launch, "launches": tm["mlp_launches"],
                  "share_of_wall": mlp_ms * 1e-3 / el}
    for v in out.values():
        v["frac"] = v["achieved"] / v["peak"]
    dom = "movegen" if mg_ms >= mlp_ms else "mlp"
    r = {k: out[dom][k] for k in ("bound", "achieved", "peak", "unit", "frac")}
    r["kernel"] = (("movegen launch = bgx::movegen_few_kernel + bgx::movegen_block_kernel" if leg == "1ply" else
                    "movegen launches = (few | pool) + bgx::movegen_block_kernel")
                   if dom == "movegen" else "bgx::mlp_kernel")
    r["traffic"], r["traffic_source"] = (_pmc(leg, dom, "hbm_bytes_per_launch", lanes) if leg != "1ply"
                                         else (None, None))
    if r["traffic"]:
        r["physical_gbs"] = r["traffic"] / (out[dom]["avg_launch_ms"] * 1e-3) / 1e9
    for key in ("valu_busy", "mfma_busy", "wait_frac", "issue_stall_frac", "waves_per_cu"):
        v, _src = _pmc(leg, dom, key, lanes) if leg != "1ply" else (None, None)
        if v is not None:
            r[key] = v
    return r, out


def spawn_ranks(n):
    """bench.py --gpus N without a torch.distributed launcher: start the N
    rank processes through torch.distributed.run from this process, which
    has not touched a GPU, and exit with their status."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps of the headline leg (the driver passes it: one run at --seed). Without it, "
                         "SURVEY 8d's protocol: every leg over seeds 0-4, each with a timed window of >= "
                         "--window-s seconds, the median reported")
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--window-s", type=float, default=10.0, help="protocol mode: timed seconds per leg and seed")
    ap.add_argument("--seeds", type=int, default=5, help="protocol mode: seeds 0..n-1")
    ap.add_argument("--lanes", type=int, default=8192,
                    help="lanes per GPU (8,192: configs[3]/[4]'s 65,536 lanes over 8 GPUs)")
    ap.add_argument("--ply", type=int, default=1)
    ap.add_argument("--k-top", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--desync-steps", type=int, default=300,
                    help="untimed steps before the warmup so lanes are spread over their games (SURVEY 8d)")
    ap.add_argument("--desync-ms", type=float, default=50.0,
                    help="... and at least this much GPU time (more chunks of --harvest-every steps), so the "
                         "window does not start on a GPU that idled through the CPU baseline")
    ap.add_argument("--harvest-every", type=int, default=300,
                    help="steps per bgx_step launch between harvests (<= ring - max_steps)")
    ap.add_argument("--two-ply-steps", type=int, default=100, help="2-ply K=4 leg (configs[4]); 0 = skip")
    ap.add_argument("--kall-steps", type=int, default=20,
                    help="2-ply K=all leg (configs[2]: ~21 x C reply boards per decision); 0 = skip")
    ap.add_argument("--config1-steps", type=int, default=300,
                    help="N = 1: configs[1] (4,096 lanes, 1-ply) beside the headline; 0 = skip")
    ap.add_argument("--config2-steps", type=int, default=100,
                    help="N = 1: configs[2] (4,096 lanes, 2-ply) beside the headline: K=4 for this many steps, "
                         "K=all for a fifth of them; 0 = skip")
    ap.add_argument("--cpu-procs", type=int, default=7, help="pinned CPU-port processes (src/main.py:86: 7 workers)")
    ap.add_argument("--cpu-seconds", type=float, default=2.0, help="per 1-ply round (one round per seed)")
    ap.add_argument("--cpu-seeds", type=int, default=5, help="seeds 0..n-1, median reported")
    ap.add_argument("--cpu-2ply-seconds", type=float, default=4.0, help="2-ply CPU round (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fused", action="store_true",
                    help="1-ply: one launch per phase and step instead of the fused persistent step kernel")
    ap.add_argument("--gather", choices=("host", "device", "rccl"), default="host",
                    help="N > 1 episode gather to rank 0: 'host' = DMA-engine copies into host shared memory "
                         "(no kernels, no collective per harvest); 'device' = DMA-engine peer copies into rank 0's "
                         "GPU memory (xGMI, the GPU trainer's input); 'rccl' = RCCL point-to-point over xGMI")
    ap.add_argument("--collect-copy", action="store_true",
                    help="N > 1: rank 0 clones each gathered batch on its GPU (devgather.collect(copy=True), the "
                         "GPU trainer's input) instead of reading the slots in place")
    ap.add_argument("--no-balance", action="store_true",
                    help="fused 1-ply: every lane runs exactly the steps of a call (lockstep) instead of the "
                         "balanced launch (a step(n) call = n x lanes lane-steps, faster workgroups run ahead)")
    ap.add_argument("--timing-steps", type=int, default=200,
                    help="length of the event-timed pass that feeds roofline (2-ply: min(this, 50))")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world_env = int(os.environ.get("WORLD_SIZE", "1"))

    # the CPU baseline first, on rank 0 at N = 1, before this process touches the GPU
    cpu = None
    if world_env == 1 and not args.no_cpu_baseline:
        r = cpu_baseline(args.cpu_procs, args.cpu_seconds, list(range(args.cpu_seeds)), args.cpu_2ply_seconds)
        cpu = {"value": r["1ply"]["median"], "unit": "env_steps/s", "cores": r["cores_used"], "kind": "port",
               "sample": (f"{args.cpu_procs} processes, each pinned to one host core, x {args.cpu_seconds:.0f} s "
                          f"of 1-ply self-play per seed after a {CPU_WARMUP_STEPS}-step warm-up (seeds 0-{args.cpu_seeds - 1}, median of "
                          f"{[round(x) for x in r['1ply']['rates']]}) with the CPU port of the worker loop "
                          f"(oracle/bgref.c; same weights, T=1.5); host: {r['cpu_model']}, nproc {r['nproc']}, "
                          f"{r['affinity']} cores in this process's affinity mask; the reference's own Python "
                          f"7-worker path measured 2,052 env steps/s in the survey container (BASELINE.md)"),
               "cpu_model": r["cpu_model"], "nproc": r["nproc"]}
        if "2ply" in r:
            cpu["two_ply_k4"] = {"value": r["2ply"]["value"], "unit": "env_steps/s",
                                 "decisions_per_s": r["2ply"]["decisions_per_s"],
                                 "sample": f"{args.cpu_procs} pinned processes x {r['2ply']['elapsed']:.1f} s of "
                                           f"2-ply K=4 self-play (exact mode, fp32) with the same CPU port, each "
                                           f"after a {CPU_WARMUP_STEPS}-step warm-up of 1-ply decisions that ends "
                                           "mid-game (the window starts from the self-play position mix); the "
                                           "reference's Python 2-ply takes 205 ms per decision (BASELINE.md)"}

    world, rank, local = init_dist()

    def leg(ply, k_top, lanes, steps, warmup, timing_steps, name, desync=None, seed=None):
        desync = args.desync_steps if desync is None else desync
        el_, d_, tm_, dtm_, gathered_, harvested_ = run_engine(args, world, rank, ply, k_top, lanes, steps, warmup,
                                                   args.harvest_every, timing=timing_steps > 0,
                                                   timing_steps=timing_steps, desync=desync, seed=seed)
        el_ = max_over_ranks(el_, world)
        per_rank = [int(x) for x in all_ranks(d_["env_steps"], world)]
        roof_, kern_ = roofline_for(dtm_, tm_, name, lanes) if timing_steps > 0 else (None, None)
        out_ = {"value": sum(per_rank) / el_, "unit": "env_steps/s", "steps": steps, "lanes_per_gpu": lanes,
                "ms_per_step": el_ / steps * 1e3, "env_steps_per_rank": per_rank,
                "decisions_per_s": sum_over_ranks(d_["decisions"], world) / el_,
                "episodes_per_s": sum_over_ranks(d_["episodes"], world) / el_,
                "value_rows_per_s": sum_over_ranks(d_["value_rows"], world) / el_,
                "movegen_jobs_per_s": sum_over_ranks(d_["movegen_jobs"], world) / el_,
                "fallback_jobs": int(sum_over_ranks(d_["fallback_jobs"], world)),
                # 2-ply: reply rows the movegen reserved but left unwritten (the MLP
                # evaluates them; the algorithmic figures below leave them out)
                "gap_rows_frac": sum_over_ranks(d_["gap_rows"], world) / max(1, sum_over_ranks(d_["value_rows"], world)),
                "roofline": roof_, "kernels": kern_, "desync_steps": int(d_.get("desync_steps_run", desync)),
                "seed": args.seed if seed is None else seed}
        if world > 1:
            out_["gathered_episodes"], out_["gathered_records"] = gathered_
            if rank == 0 and d_.get("collect_batches"):   # rank 0's time in collect() per batch vs the interval
                out_["collect_ms_per_batch"] = d_["collect_s"] / d_["collect_batches"] * 1e3
                out_["harvest_interval_ms"] = el_ / d_["collect_batches"] * 1e3
            # what each rank harvested (all of the engine's runs, as the gather counts)
            out_["harvested_episodes_per_rank"] = [int(x) for x in all_ranks(harvested_[0], world)]
            out_["harvested_records_per_rank"] = [int(x) for x in all_ranks(harvested_[1], world)]
        if rank == 0:   # progress on stderr (the JSON line is stdout's only line)
            print(f"[bench] {name} lanes={lanes} seed={out_['seed']} steps={steps}: {out_['value'] / 1e6:.2f} M env "
                  f"steps/s, {out_['ms_per_step']:.4f} ms/step", file=sys.stderr, flush=True)
        return out_, d_

    def protocol(ply, k_top, lanes, warmup, timing_steps, name, short_steps):
        """seeds 0..n-1, each a fresh engine with a timed window of
        >= --window-s seconds (steps sized from a short calibration run of
        seed 0), the median by value reported with every seed's figures."""
        cal, _ = leg(ply, k_top, lanes, short_steps, warmup, 0, name, seed=0)
        per = args.harvest_every
        steps = max(short_steps, -(-int(args.window_s * 1e3 / cal["ms_per_step"]) // per) * per)
        runs = []
        for sd in range(args.seeds):
            r, d_ = leg(ply, k_top, lanes, steps, warmup, timing_steps if sd == 0 else 0, name, seed=sd)
            runs.append((r, d_))
        order = sorted(range(len(runs)), key=lambda i: runs[i][0]["value"])
        med, dmed = runs[order[len(runs) // 2]]
        med = dict(med)
        med["roofline"], med["kernels"] = runs[0][0]["roofline"], runs[0][0]["kernels"]   # seed 0's timing pass
        med["protocol"] = {"seeds": [r["seed"] for r, _ in runs], "values": [r["value"] for r, _ in runs],
                           "ms_per_step": [r["ms_per_step"] for r, _ in runs], "steps_per_seed": steps,
                           "window_s": [r["ms_per_step"] * steps * 1e-3 for r, _ in runs],
                           "median_seed": med["seed"], "calibration_steps": short_steps}
        return med, dmed

    proto = args.steps is None
    head_name = "1ply" if args.ply == 1 else ("2ply_k4" if args.k_top == 4 else "2ply_kall")
    if proto:
        head, d = protocol(args.ply, args.k_top, args.lanes, args.warmup, args.timing_steps, head_name, 1200)
        args.steps = head["steps"]
    else:
        head, d = leg(args.ply, args.k_top, args.lanes, args.steps, args.warmup, min(args.steps, args.timing_steps),
                      head_name)
    extra = {}
    if args.ply == 1 and args.two_ply_steps > 0:
        extra["two_ply_k4"], _ = (protocol(2, 4, args.lanes, 20, min(args.timing_steps, 50), "2ply_k4", 100)
                                  if proto else
                                  leg(2, 4, args.lanes, args.two_ply_steps, 20,
                                      min(args.two_ply_steps, args.timing_steps, 50), "2ply_k4"))
    if args.ply == 1 and args.kall_steps > 0:
        extra["two_ply_kall"], d3 = (protocol(2, 0, args.lanes, 5, min(args.timing_steps, 10), "2ply_kall", 20)
                                     if proto else
                                     leg(2, 0, args.lanes, args.kall_steps, 5,
                                         min(args.kall_steps, args.timing_steps, 10), "2ply_kall"))
        extra["two_ply_kall"]["reply_boards_per_decision"] = \
            (d3["value_rows"] - d3["gap_rows"] - 2 * d3["env_steps"]) / max(1, d3["decisions"])
    if args.ply == 1 and world == 1 and args.config1_steps > 0 and args.lanes != 4096:
        c1, _ = (protocol(1, 4, 4096, 100, min(args.config1_steps, args.timing_steps), "1ply", 600) if proto else
                 leg(1, 4, 4096, args.config1_steps, 100, min(args.config1_steps, args.timing_steps), "1ply"))
        extra["configs1_4096_lanes"] = {k: c1[k] for k in ("value", "unit", "steps", "ms_per_step", "roofline")
                                        + (("protocol",) if proto else ())}
    if args.ply == 1 and world == 1 and args.config2_steps > 0 and args.lanes != 4096:
        # configs[2]: 4,096 lanes, 2-ply on one MI355X (its "~21^2 next-boards/step" is K=all; K=4 is the
        # reference's two_ply.py:67-70 default), both legs at that lane count
        keys = ("value", "unit", "steps", "ms_per_step", "decisions_per_s", "gap_rows_frac", "roofline", "kernels")
        c2 = {}
        for name, k_top, n, wu in (("2ply_k4", 4, args.config2_steps, 20),
                                   ("2ply_kall", 0, max(5, args.config2_steps // 5), 5)):
            r, _ = (protocol(2, k_top, 4096, wu, min(args.timing_steps, 50 if k_top else 10), name, n) if proto else
                    leg(2, k_top, 4096, n, wu, min(n, args.timing_steps, 50 if k_top else 10), name))
            c2[name.replace("2ply_", "two_ply_")] = {k: r[k] for k in keys + (("protocol",) if proto else ())}
        extra["configs2_4096_lanes"] = c2

    if rank == 0:
        line = {
            "metric": METRIC, "value": head["value"], "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8 game state + fp16x2-split MFMA (fp32 acc)",
            "data": "synthetic: random-seeded self-play from the reference reset, seeded xavier weights",
            "config": {"workload": (f"{args.lanes} game lanes per GPU ({args.lanes * world} total), "
                                    f"{args.ply}-ply" + (" softmax select" if args.ply == 1 else
                                                        f" K={args.k_top or 'all'}")
                                    + (" (configs[3]/[4] lane shard: 65,536 lanes at N=8)"
                                       if args.lanes == 8192 else "")),
                       "lanes_per_gpu": args.lanes, "lanes_total": args.lanes * world, "ply": args.ply,
                       "harvest_every": args.harvest_every,
                       "engine": ("fused step kernel" + ("" if args.no_balance else ", balanced launches")
                                  if args.ply == 1 and not args.no_fused else "phased launches"),
                       "parallelism": ((f"lanes sharded x{world}, episode gather to rank 0 over the DMA engines "
                                        f"into page-locked host memory (memfd segments)" if args.gather == "host"
                                        else f"lanes sharded x{world}, episode gather over the DMA engines into "
                                        f"rank 0's GPU memory (IPC, xGMI peer copies)" if args.gather == "device"
                                        else f"lanes sharded x{world}, RCCL episode gather to rank 0 ({BACKEND})")
                                       if world > 1 else "single GPU")},
            "desync_steps": head["desync_steps"],
            "world_size": world, "env_steps_per_rank": head["env_steps_per_rank"],
            "decisions_per_s": head["decisions_per_s"], "episodes_per_s": head["episodes_per_s"],
            "value_rows_per_s": head["value_rows_per_s"], "fallback_jobs": head["fallback_jobs"],
            "gap_rows_frac": head["gap_rows_frac"],
            "roofline": head["roofline"], "kernels": head["kernels"], "cpu_baseline": cpu,
            "seed": head["seed"], "protocol": head.get("protocol"),
            "episodes_per_s_note": "device-side: episodes finished and harvested on the GPU per second"
                                   + (" (at N = 1 nothing is moved off the device inside the timed region)"
                                      if world == 1 else ""),
        }
        if world > 1:
            for k in ("gathered_episodes", "gathered_records", "harvested_episodes_per_rank",
                      "harvested_records_per_rank", "collect_ms_per_batch", "harvest_interval_ms"):
                if k in head:
                    line[k] = head[k]
        line.update(extra)
        print(json.dumps(line))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
