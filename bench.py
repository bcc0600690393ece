#!/usr/bin/env python3
"""Self-play throughput benchmark (BASELINE.json metric: self-play env steps/sec).

One bench "step" = one env step (one BackgammonEnv.step equivalent, passes
included) of every lane on every GPU, including the compact Experience
records, the episode harvest (every --harvest-every steps) and, for N > 1,
the RCCL gather of the harvested episodes to rank 0. Synthetic data: lanes
start from the reference's reset and play random-seeded self-play with the
seeded xavier weights (tests/golden/weights_seed0.npz = torch.manual_seed(0)
BackgammonPolicyNetwork()), T = 1.5 (ParameterManager version 1).

N = 1:  python bench.py
N > 1:  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
            --master-addr 127.0.0.1 --master-port P bench.py --gpus N
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
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


def sum_over_ranks(x, world):
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=_coll_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def run_engine(args, world, rank, ply, k_top, lanes, steps, warmup, harvest_every, timing, timing_steps=0):
    from bgx import Engine
    from bgx import dist as bdist
    w = load_weights()
    if world > 1:
        w = bdist.broadcast_weights(w)
    eng = Engine(lanes=lanes, seed=args.seed, ply=ply, k_top=k_top, lane_base=rank * lanes,
                 fused=not args.no_fused)
    eng.set_weights(w, temperature=1.5, version=1)
    gathered = [0, 0]

    def run(n):
        # the gather of a harvest stays in flight while the next steps run and
        # is waited at the next harvest (or the end of the run)
        left, pending = n, None

        def collect(p):
            eps, recs = p.wait()
            if rank == 0:
                gathered[0] += eps
                gathered[1] += recs

        while left > 0:
            k = min(harvest_every, left)
            eng.step(k)
            h = eng.harvest()
            if world > 1:
                if pending is not None:
                    collect(pending)
                pending = bdist.gather_episodes(h, dst=0, async_op=True)
            left -= k
        if pending is not None:
            collect(pending)

    run(warmup)
    eng.sync()
    s0 = eng.stats()
    barrier(world)
    t0 = time.perf_counter()
    run(steps)          # graph-launched step sequence, no events in the stream
    barrier(world)
    el = time.perf_counter() - t0
    s1 = eng.stats()
    d = {k: s1[k] - s0[k] for k in s1}
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
    return el, d, tm, d_tm, gathered


def cpu_baseline(seconds, threads):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc  # the bench's cpu_baseline leg (oracle = the CPU port)
    r = orc.selfplay_bench(load_weights(), temperature=1.5, seed=0, n_threads=threads, seconds=seconds)
    return r


def roofline_fused(d, tm):
    """The fused 1-ply step kernel (one launch = all steps of a step() call):
    the whole path's algorithmic bytes (54 B per movegen job +
    901 B per evaluated board) and MLP FLOPs over its average launch."""
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
    r = {kk: k[kk] for kk in ("bound", "achieved", "peak", "unit", "frac")}
    r["kernel"] = "bgx::fused_step_kernel (movegen + encode + MLP + select + env step, all steps of a launch)"
    r["traffic"] = None
    prof = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                per_step = json.load(f).get("1ply_fused", {}).get("fused", {}).get("hbm_bytes_per_step")
                # PMC bytes per step (tools/profile_round.sh) x the steps of this bench's launches
                r["traffic"] = per_step * k["steps_per_launch"] if per_step else None
        except Exception:
            r["traffic"] = None
    return r, {"fused_step": k, "fused_step_mfma": m}


def roofline_for(d, tm, leg):
    """Dominant kernel's algorithmic rate over its average launch (HIP events),
    from the timed pass `d` (stats deltas) / `tm` (event totals)."""
    if tm["mlp_launches"] == 0 and tm["movegen_launches"] > 0:
        return roofline_fused(d, tm)
    el = d["elapsed_s"]
    mg_ms, mlp_ms = tm["movegen_ms"], tm["mlp_ms"]
    out = {}
    # boards movegen wrote = value rows minus the lanes' own rows (one per lane step)
    mg_rows = d["value_rows"] - d["env_steps"]
    mg_bytes = MOVEGEN_BYTES_PER_JOB * d["movegen_jobs"] + MOVEGEN_BYTES_PER_ROW * mg_rows
    mg_launch = mg_ms / max(1, tm["movegen_launches"])
    out["movegen"] = {"bound": "hbm", "achieved": mg_bytes / max(1, tm["movegen_launches"]) / (mg_launch * 1e-3) / 1e9,
                      "peak": HBM_PEAK_GBS, "unit": "GB/s", "avg_launch_ms": mg_launch,
                      "launches": tm["movegen_launches"], "share_of_wall": mg_ms * 1e-3 / el}
    mlp_launch = mlp_ms / max(1, tm["mlp_launches"])
    mlp_flop = MLP_FLOP_PER_ROW * d["value_rows"] / max(1, tm["mlp_launches"])
    out["mlp"] = {"bound": "mfma", "achieved": mlp_flop / (mlp_launch * 1e-3) / 1e12, "peak": FP16_DENSE_PEAK_TFS,
                  "unit": "TFLOP/s", "avg_launch_ms": mlp_launch, "launches": tm["mlp_launches"],
                  "share_of_wall": mlp_ms * 1e-3 / el}
    for v in out.values():
        v["frac"] = v["achieved"] / v["peak"]
    dom = "movegen" if mg_ms >= mlp_ms else "mlp"
    r = {k: out[dom][k] for k in ("bound", "achieved", "peak", "unit", "frac")}
    r["kernel"] = ({"1ply": "movegen launch = bgx::movegen_few_kernel + bgx::movegen_block_kernel",
                    "2ply": "movegen launches = (few | pool) + bgx::movegen_block_kernel"}[leg]
                   if dom == "movegen" else "bgx::mlp_kernel")
    r["traffic"] = None
    prof = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                r["traffic"] = json.load(f).get(leg, {}).get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            r["traffic"] = None
    return r, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=300)
    ap.add_argument("--lanes", type=int, default=4096, help="lanes per GPU (configs[1]: 4096)")
    ap.add_argument("--ply", type=int, default=1)
    ap.add_argument("--k-top", type=int, default=4)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--harvest-every", type=int, default=300,
                    help="steps per bgx_step launch between harvests (<= ring - max_steps = 340)")
    ap.add_argument("--two-ply-steps", type=int, default=100, help="extra 2-ply (K=4) measurement; 0 = skip")
    ap.add_argument("--kall-steps", type=int, default=20,
                    help="extra 2-ply K=all measurement (configs[2]: ~21 x C reply boards per decision); 0 = skip")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=7, help="mirrors src/main.py:86 (7 workers)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fused", action="store_true",
                    help="1-ply: one launch per phase and step instead of the fused persistent step kernel")
    ap.add_argument("--timing-steps", type=int, default=200,
                    help="length of the event-timed pass that feeds roofline (2-ply: min(this, 50))")
    args = ap.parse_args()

    world, rank, local = init_dist()
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    el, d, tm, d_tm, gathered = run_engine(args, world, rank, args.ply, args.k_top, args.lanes, args.steps,
                                           args.warmup, args.harvest_every, timing=True,
                                           timing_steps=min(args.steps, args.timing_steps))
    el = max_over_ranks(el, world)
    total_steps = sum_over_ranks(d["env_steps"], world)
    value = total_steps / el
    roof, kernels = roofline_for(d_tm, tm, f"{args.ply}ply")

    extra = {}
    if args.two_ply_steps > 0 and args.ply == 1:
        el2, d2, tm2, d2_tm, _ = run_engine(args, world, rank, 2, 4, args.lanes, args.two_ply_steps, 20,
                                            args.harvest_every, timing=True,
                                            timing_steps=min(args.two_ply_steps, args.timing_steps, 50))
        el2 = max_over_ranks(el2, world)
        tot2 = sum_over_ranks(d2["env_steps"], world)
        r2, k2 = roofline_for(d2_tm, tm2, "2ply")
        extra["two_ply_k4"] = {"value": tot2 / el2, "unit": "env_steps/s", "steps": args.two_ply_steps,
                               "ms_per_step": el2 / args.two_ply_steps * 1e3,
                               "value_rows_per_s": sum_over_ranks(d2["value_rows"], world) / el2,
                               "movegen_jobs_per_s": sum_over_ranks(d2["movegen_jobs"], world) / el2,
                               "roofline": r2, "kernels": k2}

    if args.kall_steps > 0 and args.ply == 1:
        el3, d3, tm3, d3_tm, _ = run_engine(args, world, rank, 2, 0, args.lanes, args.kall_steps, 5,
                                            args.harvest_every, timing=True,
                                            timing_steps=min(args.kall_steps, args.timing_steps, 10))
        el3 = max_over_ranks(el3, world)
        tot3 = sum_over_ranks(d3["env_steps"], world)
        r3, k3 = roofline_for(d3_tm, tm3, "2ply")
        r3["traffic"] = None   # the PMC passes cover the K=4 leg
        extra["two_ply_kall"] = {"value": tot3 / el3, "unit": "env_steps/s", "steps": args.kall_steps,
                                 "ms_per_step": el3 / args.kall_steps * 1e3,
                                 "value_rows_per_s": sum_over_ranks(d3["value_rows"], world) / el3,
                                 "movegen_jobs_per_s": sum_over_ranks(d3["movegen_jobs"], world) / el3,
                                 "reply_boards_per_decision": (d3["value_rows"] - 2 * d3["env_steps"])
                                 / max(1, d3["decisions"]),
                                 "roofline": r3, "kernels": k3}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        r = cpu_baseline(args.cpu_seconds, args.cpu_threads)
        cpu = {"value": r["steps"] / r["elapsed"], "unit": "env_steps/s", "cores": r["threads"], "kind": "port",
               "sample": f"{r['threads']} host threads x {r['elapsed']:.1f} s of 1-ply self-play with the CPU "
                         f"oracle port (oracle/bgref.c; same weights, T=1.5): {r['steps']} env steps, "
                         f"{r['episodes']} episodes; reference Python 7-worker path measured 2052 env steps/s "
                         f"in the survey container (BASELINE.md)"}

    sums = {k: sum_over_ranks(d[k], world) for k in ("decisions", "episodes", "value_rows", "fallback_jobs")}
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "env_steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8 game state + fp16x2-split MFMA (fp32 acc)",
            "data": "synthetic: random-seeded self-play from the reference reset, seeded xavier weights",
            "config": {"workload": f"{args.lanes} game lanes per GPU, {args.ply}-ply softmax select"
                                   + (" (configs[1])" if args.ply == 1 and args.lanes == 4096 else ""),
                       "lanes_per_gpu": args.lanes, "lanes_total": args.lanes * world, "ply": args.ply,
                       "harvest_every": args.harvest_every,
                       "engine": "fused step kernel" if args.ply == 1 and not args.no_fused else "phased launches",
                       "parallelism": f"lanes sharded x{world}, "
                       "RCCL episode gather" if world > 1 else "single GPU"},
            "decisions_per_s": sums["decisions"] / el,
            "episodes_per_s": sums["episodes"] / el,
            "value_rows_per_s": sums["value_rows"] / el,
            "fallback_jobs": int(sums["fallback_jobs"]),
            "roofline": roof, "kernels": kernels, "cpu_baseline": cpu,
        }
        if world > 1:
            line["gathered_episodes"] = gathered[0]
        line.update(extra)
        print(json.dumps(line))
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
