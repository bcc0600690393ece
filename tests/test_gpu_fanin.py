"""The N = 8 episode fan-in of bench.py, rehearsed on one GPU.

bench.py --gpus 8 as the driver's 8-GPU run starts it (torch.distributed.run,
8 rank processes), with the gloo backend so the 8 ranks can time-share
cuda:0: every rank drives its own 1,024-lane engine and 7 ranks hand their
harvests to rank 0 through the host gather (DMA-engine copies into page-locked
memfd segments, bgx/hostgather.py) -- the path of the reference's 7 workers
putting Episodes on one queue for the trainer (src/main.py:86-91, 115-133).
Checked: the JSON line reports world size 8 and one env-step count per rank,
and rank 0 gathered exactly the episodes and records the 8 ranks harvested.
A rank that fails mid-run makes the whole command exit non-zero within its
gather timeout instead of leaving rank 0 waiting."""
import json
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--gpus", "8", "--lanes", "1024", "--steps", "60", "--warmup", "10", "--desync-steps", "60",
        "--harvest-every", "30", "--two-ply-steps", "0", "--kall-steps", "0", "--config1-steps", "0",
        "--timing-steps", "0"]


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update({"BGX_DIST_BACKEND": "gloo", "HSA_ENABLE_IPC_MODE_LEGACY": "0", "BGX_GATHER_TIMEOUT": "40",
                "OMP_NUM_THREADS": "1"}, **extra)
    return env


@pytest.mark.parametrize("gather", ["host", "device-copy"])
def test_bench_world8_fanin_on_one_gpu(gather):
    """host: the default hand-off. device-copy: the device gather (slots in rank
    0's GPU memory, opened by the 7 peers over IPC, SDMA peer copies;
    bgx/devgather.py), rank 0 cloning every batch on its own stream as the GPU
    trainer takes it (collect(copy=True)); the JSON line then reports rank 0's
    time inside collect() per batch beside the harvest interval."""
    extra = ["--gather", "host"] if gather == "host" else ["--gather", "device", "--collect-copy"]
    r = subprocess.run([sys.executable, "bench.py", *ARGS, *extra], cwd=REPO, env=_env(), capture_output=True,
                       text=True, timeout=420)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 8 and line["world_size"] == 8
    assert len(line["env_steps_per_rank"]) == 8 and min(line["env_steps_per_rank"]) >= 1024 * 60
    eps, recs = line["harvested_episodes_per_rank"], line["harvested_records_per_rank"]
    assert len(eps) == 8 and min(eps) > 0
    assert line["gathered_episodes"] == sum(eps), (line["gathered_episodes"], eps)
    assert line["gathered_records"] == sum(recs), (line["gathered_records"], recs)
    assert line["collect_ms_per_batch"] >= 0 and line["harvest_interval_ms"] > 0
    print(f"[fanin {gather}] collect {line['collect_ms_per_batch']:.3f} ms per batch, harvest interval "
          f"{line['harvest_interval_ms']:.3f} ms, {line['value'] / 1e6:.2f} M env steps/s")


def test_bench_world8_failed_rank_ends_the_run():
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "bench.py", *ARGS, "--gather", "host"], cwd=REPO,
                       env=_env(BGX_BENCH_FAIL_RANK="5"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "BGX_BENCH_FAIL_RANK" in r.stderr
    assert time.monotonic() - t0 < 240
