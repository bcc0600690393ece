"""World-size-2 gloo rehearsal of the multi-GPU path (bgx.dist) on CPU:
weight broadcast from the trainer rank and the episode gather."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    from bgx import dist as bdist
    from bgx.engine import Harvest
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    w = {"W1": rng.standard_normal((128, 198)).astype(np.float32), "b1": np.full(128, rank, np.float32),
         "w2": np.ones(128, np.float32), "b2": np.array([rank], np.float32)}
    got = bdist.broadcast_weights(w, src=0)
    base, n = bdist.lane_block(rank, 4096)
    # rank r finished r+1 episodes with 3*(r+1) records, tagged with its lane block
    hdr = torch.zeros((rank + 1, 16), dtype=torch.int32)
    hdr[:, 0] = base
    rec = torch.full((3 * (rank + 1), 12), rank + 7, dtype=torch.int32)
    res = bdist.gather_episodes(Harvest(hdr, rec), dst=0, keep=True)
    # the asynchronous form (bench.py overlaps it with the next steps) returns the same
    pend = bdist.gather_episodes(Harvest(hdr, rec), dst=0, keep=True, async_op=True)
    res_a = pend.wait()
    assert res_a[:2] == res[:2]
    for (h0, r0), (h1, r1) in zip(res[2], res_a[2]):
        assert torch.equal(h0, h1) and torch.equal(r0, r1)
    if rank == 0:
        out.put(("w", got["b1"][0], got["b2"][0]))
        out.put(("tot", res[0], res[1], [int(p[0][0, 0]) for p in res[2]], [int(p[1][0, 0]) for p in res[2]]))
    else:
        out.put(("w1", got["b1"][0]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_broadcast_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=120) for _ in range(3)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = {m[0]: m[1:] for m in msgs}
    assert d["w"] == (0.0, 0.0) and d["w1"] == (0.0,)   # every rank holds rank 0's weights
    tot_eps, tot_recs, lane0, tag = d["tot"]
    assert (tot_eps, tot_recs) == (1 + 2, 3 + 6)
    assert lane0 == [0, 4096] and tag == [7, 8]


class _FakeEngine:
    def __init__(self):
        self.calls = []

    def set_weights(self, w, temperature, version):
        self.calls.append((float(w["b1"][0]), float(temperature), int(version)))


def _pm_worker(rank, world, port, out):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    from multi.parameter_manager import DistributedParameterManager
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _FakeEngine()
    sd = {"fc1.weight": torch.zeros(128, 198), "fc1.bias": torch.full((128,), 0.5),
          "value_head.weight": torch.ones(1, 128), "value_head.bias": torch.zeros(1)}
    pm = DistributedParameterManager(engine=eng, src=0, state_dict=sd if rank == 0 else None)
    first = (pm.get_version(), pm.get_temperature())
    quiet = pm.sync()                                   # nothing new: no weight broadcast
    if rank == 0:
        for k in range(3):                              # three trainer updates before one sync
            sd["fc1.bias"] = torch.full((128,), float(k + 1))
            pm.set_parameters(sd)
    moved = pm.sync()
    got = pm.get_parameters()
    out.put((rank, first, quiet, moved, pm.get_version(), pm.get_temperature(), eng.calls,
             float(got["fc1.bias"][0]), tuple(got["value_head.weight"].shape)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_distributed_parameter_manager():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {m[0]: m[1:] for m in (q.get(timeout=120) for _ in range(2))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        first, quiet, moved, ver, temp, calls, b1, w2shape = res[r]
        assert first == (1, 1.5)                        # version 1 everywhere after construction
        assert quiet is False and moved is True
        assert ver == 4 and abs(temp - (1.5 - 1.0 * 3 / 4000)) < 1e-12   # parameter_manager.py:101-111
        assert calls == [(0.5, 1.5, 1), (3.0, temp, 4)]  # engine re-armed once per propagated version
        assert b1 == 3.0 and w2shape == (1, 128)


def _hg_worker(rank, world, port, out):
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    import torch.distributed as dist
    from bgx import hostgather
    from bgx.engine import Harvest
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = hostgather.setup(rank, world, slot_bytes=1 << 16, dst=0)
    got = []
    for seq in range(1, 6):
        # rank r's batch seq: (r + seq) % 3 episodes (some empty), 2 records each
        ne = (rank + seq) % 3
        hdr = torch.full((ne, 16), 1000 * rank + seq, dtype=torch.int32)
        rec = torch.arange(2 * ne * 12, dtype=torch.int32).view(-1, 12) + 100 * seq
        if rank == 0:
            parts = g.collect(seq)
            got.append([None if p is None else (p[0].copy(), p[1].copy()) for p in parts])
        else:
            g.publish(Harvest(hdr, rec)).wait()
    if rank == 0:
        out.put(got)
    dist.barrier()
    g.close()
    dist.destroy_process_group()


def test_gloo_world3_host_gather():
    """bgx.hostgather: ranks hand their harvests to rank 0 through host shared
    memory (the DMA-engine path of bench.py --gather host; here CPU tensors),
    double-buffered, empty batches included, exact bytes, no collective per
    batch (ranks 1 and 2 may run a batch ahead of rank 0's reads)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hg_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len(got) == 5
    for seq, parts in enumerate(got, start=1):
        assert parts[0] is None
        for r in (1, 2):
            hdr, rec = parts[r]
            ne = (r + seq) % 3
            assert hdr.shape == (ne, 16) and rec.shape == (2 * ne, 12)
            assert np.all(hdr == 1000 * r + seq)
            np.testing.assert_array_equal(rec.reshape(-1), np.arange(2 * ne * 12) + 100 * seq)


def test_host_gather_segments_do_not_use_dev_shm():
    """bench.py's host gather keeps its segments in anonymous memory files
    (memfd), so the path --gpus 8 takes does not depend on /dev/shm's size (a
    container's tmpfs is often 64 MB; a rank's segment at 8,192 lanes is
    ~0.5 GB): a segment larger than /dev/shm's free space is created and its
    last page written, and nothing appears under /dev/shm."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from bgx import hostgather
    slot = hostgather.slot_bytes_for(8192, 300)
    assert slot >= 8192 * 600 * 48   # a record per lane-step since the last harvest + the open episodes
    st = os.statvfs("/dev/shm")
    free = st.f_bavail * st.f_frsize
    before = set(os.listdir("/dev/shm"))
    g = hostgather.HostGather(1, 2, hostgather.make_tag(), slot_bytes=free // 2 + (1 << 20))
    try:
        assert g._mine.size > free
        g._mine.buf[g._mine.size - 1] = 7            # a sparse file: only the touched page is backed
        assert g._mine.buf[g._mine.size - 1] == 7
        assert not any("bgx_hg" in n for n in set(os.listdir("/dev/shm")) - before)
    finally:
        g.close()


def test_host_gather_oversized_harvest_keeps_batch_numbers():
    """A harvest larger than the slot raises before the batch number moves
    (ADVICE r3): the rank can still publish the batch dst waits for."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from bgx import hostgather
    from bgx.engine import Harvest
    g = hostgather.HostGather(1, 2, hostgather.make_tag(), slot_bytes=4096)
    try:
        big = Harvest(torch.zeros((1, 16), dtype=torch.int32), torch.zeros((100, 12), dtype=torch.int32))
        with pytest.raises(ValueError):
            g.publish(big)
        assert g.seq == 0
        p = g.publish(Harvest(torch.ones((1, 16), dtype=torch.int32), torch.ones((2, 12), dtype=torch.int32)))
        assert p.wait() == 1 and int(g.ctrl[1][0]) == 1
    finally:
        g.close()


def test_host_gather_refuses_publish_before_wait():
    """A batch is published by its Pending.wait(): a second publish before it
    would move the batch number past a batch whose counts were never written,
    and dst would read that slot with the counts of the batch before it (the
    round-5 fan-in rehearsal lost 1,315 of 7,657 episodes that way in
    bench.py). The gather refuses it."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from bgx import hostgather
    from bgx.engine import Harvest
    g = hostgather.HostGather(1, 2, hostgather.make_tag(), slot_bytes=4096)
    try:
        h = Harvest(torch.ones((1, 16), dtype=torch.int32), torch.ones((2, 12), dtype=torch.int32))
        p = g.publish(h)
        with pytest.raises(RuntimeError, match="not waited"):
            g.publish(h)
        assert p.wait() == 1 and int(g.ctrl[1][0]) == 1
        g.ctrl[1][5] = 1
        assert g.publish(h).wait() == 2
    finally:
        g.close()


def test_gather_keeps_a_timed_out_copy(monkeypatch):
    """A DMA copy that did not finish within its wait (bgx_dma_wait returns
    BGX_E_STATE and leaves it in flight): the batch is not published, its
    source arrays stay referenced for the life of the process, and the gather
    refuses further batches instead of reusing a slot a DMA engine may still
    write."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from bgx import _lib, hostgather
    from bgx.engine import Harvest

    class Fake:
        def bgx_dma_wait(self, ticket, timeout_ms):
            return -5

        def bgx_last_error(self):
            return b"bgx_dma_wait: copy not finished after 1 ms"

    monkeypatch.setattr(_lib, "_lib", Fake())
    g = hostgather.HostGather(1, 2, hostgather.make_tag(), slot_bytes=4096)
    try:
        keep = (torch.ones((1, 16), dtype=torch.int32), torch.ones((2, 12), dtype=torch.int32))
        p = hostgather.Pending(g, 1, 1, 2, 1, None, dma=(123, 456), keep=keep)
        with pytest.raises(_lib.BgxError, match="not finished"):
            p.wait()
        assert g.broken and p in hostgather.STUCK_COPIES and p.keep is keep
        assert int(g.ctrl[1][0]) == 0   # never published
        with pytest.raises(RuntimeError, match="did not finish"):
            g.publish(Harvest(*keep))
        hostgather.STUCK_COPIES.remove(p)
    finally:
        g.close()


def test_device_gather_finds_the_trainer_gpu_by_pci_location():
    """bgx/devgather.py hands the trainer rank's GPU to its peers as a PCI
    location, resolved in each peer's own device list: a location
    no visible device has is an error that names it, not a copy to whatever
    GPU shares the ordinal."""
    import sys
    from conftest import PKG
    sys.path.insert(0, PKG)
    from bgx import devgather
    with pytest.raises(RuntimeError, match="0000:c3:00"):
        devgather.device_by_pci((0, 0xC3, 0))
