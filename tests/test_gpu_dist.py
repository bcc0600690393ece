"""The multi-GPU path with real engines: two ranks (gloo, both on cuda:0 --
the rehearsal form of bench.py's one-process-per-GPU run) each drive an
Engine over their lane block and gather their REAL harvests to rank 0
(bgx.dist.gather_episodes); rank 0 checks them against one Engine over both
blocks: same episodes, same records (src/main.py:86-91 spreads the games over
worker processes; here over GPUs, with RCCL in place of gloo on a node)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, L, steps, out):
    import sys
    from conftest import PKG, golden
    sys.path.insert(0, PKG)
    import torch
    import torch.distributed as dist
    from bgx import Engine
    from bgx import dist as bdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w = {k: golden("weights_seed0.npz")[k] for k in ("W1", "b1", "w2", "b2")}
    w = bdist.broadcast_weights(w, src=0)
    base, n = bdist.lane_block(rank, L)
    e = Engine(lanes=n, lane_base=base, seed=17)
    e.set_weights(w, 1.5, 1)
    got = []
    for chunk in (steps // 2, steps - steps // 2):
        e.step(chunk)
        h = e.harvest()
        res = bdist.gather_episodes(h, dst=0, keep=True, async_op=True).wait()
        if rank == 0:
            got.append([(hh.cpu().numpy().view(np.uint32), rr.cpu().numpy().view(np.uint32)) for hh, rr in res[2]])
    e.close()
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_gathers_real_harvests(weights_seed0):
    import torch
    from bgx import Engine
    from bgx.records import episode_bounds
    L, steps = 128, 240
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, L, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # one engine over both lane blocks, same harvest cadence
    e = Engine(lanes=2 * L, seed=17)
    e.set_weights(weights_seed0, 1.5, 1)
    want = []
    for chunk in (steps // 2, steps - steps // 2):
        e.step(chunk)
        h = e.harvest()
        want.append((h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32)))
    e.close()

    def by_episode(hdr, rec):
        offs, _ = episode_bounds(hdr)
        return {(int(r[0]), int(r[1])): (r.copy(), rec[offs[i]:offs[i + 1]]) for i, r in enumerate(hdr)}

    total = 0
    for parts, (wh, wr) in zip(got, want):
        merged = {}
        for r, (hh, rr) in enumerate(parts):
            assert np.all((hh[:, 0] >= r * L) & (hh[:, 0] < (r + 1) * L))   # each rank's lane block
            merged.update(by_episode(hh, rr))
        ref = by_episode(wh, wr)
        assert merged.keys() == ref.keys() and len(ref) > 20
        for key in ref:
            np.testing.assert_array_equal(merged[key][0], ref[key][0], err_msg=str(key))
            np.testing.assert_array_equal(merged[key][1], ref[key][1], err_msg=str(key))
        total += len(ref)
    assert total > 100


def _hg_rank(rank, world, port, L, steps, out, mode="host", chunks=None, busy=False):
    import sys
    from conftest import PKG, golden
    sys.path.insert(0, PKG)
    import torch
    import torch.distributed as dist
    from bgx import Engine, devgather, hostgather
    from bgx import dist as bdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mod = hostgather if mode == "host" else devgather
    g = mod.setup(rank, world, hostgather.slot_bytes_for(L, steps), dst=0, device=0)
    w = {k: golden("weights_seed0.npz")[k] for k in ("W1", "b1", "w2", "b2")}
    base, n = bdist.lane_block(rank, L)
    e = Engine(lanes=n, lane_base=base, seed=17)
    e.set_weights(w, 1.5, 1)
    got, pend = [], None
    for seq, chunk in enumerate(chunks or (steps // 2, steps - steps // 2), start=1):
        e.step(chunk)
        h = e.harvest()
        if rank == 0:
            if busy:
                # rank 0's stream busy when it collects: the slot clones queue behind
                # ~30 ms of work, and the peer may overwrite a slot only after they ran
                try:
                    torch.cuda._sleep(80_000_000)
                except (AttributeError, RuntimeError):
                    a = torch.ones((4096, 4096), device="cuda")
                    for _ in range(20):
                        a = (a @ a) * 0.0
            parts = g.collect(seq)
            if mode == "device":   # device tensors on rank 0's GPU
                assert all(p is None or (p[0].is_cuda and p[1].is_cuda) for p in parts)
                parts = devgather.as_numpy(parts)
            parts[0] = (h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32))
            got.append(parts)
        else:
            # DMA-engine copy into the segment; the Harvest is dropped at once and
            # its blocks are asked for again before the copy is waited for: the
            # Pending keeps them, so rank 0 still gets intact records
            p = g.publish(h)
            del h
            junk = [torch.full((1 << 20,), -1, dtype=torch.int32, device="cuda") for _ in range(16)]
            p.wait()
            del junk
    e.close()
    if rank == 0:
        out.put(got)
    dist.barrier()
    g.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["host", "device"])
def test_host_gather_world2_real_harvests(weights_seed0, mode):
    """bench.py --gather host (the path bench.py --gpus N takes, whatever
    /dev/shm holds) with real engines: two ranks on cuda:0, rank 1's harvests
    reach rank 0 through page-locked anonymous shared memory (memfd segments
    handed over by SCM_RIGHTS) by the SDMA engines (bgx_dma_copy_d2h); merged
    == one Engine over both lane blocks. mode "device" (bench.py --gather
    device, bgx/devgather.py): rank 1 copies into slots on rank 0's GPU memory,
    opened by IPC, with bgx_dma_copy_d2d; rank 0 gets device tensors. The
    device mode runs 6 batches (each of the two slots per rank reused three
    times) with rank 0's stream kept busy while it collects, so a slot
    acknowledged before its clone ran would be overwritten."""
    from bgx import Engine
    from bgx.records import episode_bounds
    L, steps = 128, 240
    chunks = (40,) * 6 if mode == "device" else None   # device: 6 batches, each slot reused three times
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hg_rank, args=(r, 2, port, L, steps, q, mode, chunks, mode == "device"))
             for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    e = Engine(lanes=2 * L, seed=17)
    e.set_weights(weights_seed0, 1.5, 1)
    want = []
    for chunk in chunks or (steps // 2, steps - steps // 2):
        e.step(chunk)
        h = e.harvest()
        want.append((h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32)))
    e.close()

    def by_episode(hdr, rec):
        offs, _ = episode_bounds(hdr)
        return {(int(r[0]), int(r[1])): (r.copy(), rec[offs[i]:offs[i + 1]]) for i, r in enumerate(hdr)}

    assert len(got) == len(want)
    total = 0
    for parts, (wh, wr) in zip(got, want):
        merged = {}
        for hh, rr in parts:
            merged.update(by_episode(hh, rr))
        ref = by_episode(wh, wr)
        assert merged.keys() == ref.keys()
        total += len(ref)
        for key in ref:
            np.testing.assert_array_equal(merged[key][0], ref[key][0], err_msg=str(key))
            np.testing.assert_array_equal(merged[key][1], ref[key][1], err_msg=str(key))
    assert total > 40   # games end from ~50 steps: the later batches hold the episodes


def _nccl_rank(rank, world, port, L, steps, out):
    import sys
    from conftest import PKG, golden
    sys.path.insert(0, PKG)
    import torch
    import torch.distributed as dist
    from bgx import Engine
    from bgx import dist as bdist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    w = {k: golden("weights_seed0.npz")[k] for k in ("W1", "b1", "w2", "b2")}
    w = bdist.broadcast_weights(w, src=0)
    base, n = bdist.lane_block(rank, L)
    e = Engine(lanes=n, lane_base=base, seed=17)
    e.set_weights(w, 1.5, 1)
    e.step(steps)
    h = e.harvest()
    if rank == 1:   # a rank with nothing to send: the gather skips its point-to-point ops
        from bgx.engine import Harvest
        h = Harvest(h.headers[:0], h.records[:0])
    res = bdist.gather_episodes(h, dst=0, keep=True, async_op=True).wait()
    if rank == 0:
        out.put([(hh.cpu().numpy().view(np.uint32), rr.cpu().numpy().view(np.uint32)) for hh, rr in res[2]])
    e.close()
    dist.barrier()
    dist.destroy_process_group()


def test_nccl_world2_gather_with_an_empty_rank(weights_seed0):
    """The RCCL (nccl backend) branch of bgx.dist.gather_episodes on two GPUs,
    device-side counts and buffers, with one rank sending nothing.
    Needs >= 2 visible GPUs (the driver's 8-GPU node); skipped on one."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    from bgx import Engine
    L, steps = 128, 120
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_nccl_rank, args=(r, 2, port, L, steps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    e = Engine(lanes=L, seed=17)   # rank 0's lane block on its own
    e.set_weights(weights_seed0, 1.5, 1)
    e.step(steps)
    h = e.harvest()
    e.close()
    assert len(got) == 2 and got[1][0].shape[0] == 0 and got[1][1].shape[0] == 0
    np.testing.assert_array_equal(got[0][0], h.headers.cpu().numpy().view(np.uint32))
    np.testing.assert_array_equal(got[0][1], h.records.cpu().numpy().view(np.uint32))
