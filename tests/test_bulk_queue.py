"""Bulk Episode path: the shared-memory ring and the
ExperienceQueue's put_records / get_records surface, across processes (CPU)."""
import multiprocessing as mp
import queue

import numpy as np
import pytest

from multi.experience_queue import ExperienceQueue, pack_message, unpack_message
from multi.shm_ring import ShmRing


def _payload(tag, i, n):
    rng = np.random.default_rng(1000 * tag + i)
    return np.concatenate([np.array([tag, i, n], np.uint32), rng.integers(0, 2**32, n, dtype=np.uint32)])


def test_ring_round_trip_with_wrap():
    ring = ShmRing(4096)
    try:
        rng = np.random.default_rng(0)
        sent = []
        got = []
        for i in range(300):
            n = int(rng.integers(0, 200))
            p = _payload(0, i, n)
            assert ring.put(p.tobytes(), n_episodes=1, timeout=1.0)
            sent.append(p)
            if rng.random() < 0.6 or ring.pending_messages > 5:
                while ring.pending_messages:
                    b, ne = ring.get(timeout=1.0)
                    assert ne == 1
                    got.append(np.frombuffer(b, np.uint32))
        while ring.pending_messages:
            got.append(np.frombuffer(ring.get(timeout=1.0)[0], np.uint32))
        assert len(got) == len(sent)
        for a, b in zip(sent, got):
            np.testing.assert_array_equal(a, b)
        assert ring.get(timeout=0.01) is None
        assert ring.pending_episodes == 0
    finally:
        ring.close()


def test_ring_rejects_oversize_and_times_out_when_full():
    ring = ShmRing(1024)
    try:
        with pytest.raises(ValueError):
            ring.put(bytes(2048))
        assert ring.put(bytes(600), timeout=0.1)
        assert not ring.put(bytes(600), timeout=0.05)   # full: the consumer has not read
        assert ring.get(timeout=0.1)[0] == bytes(600)
        assert ring.put(bytes(600), timeout=0.1)
    finally:
        ring.close()


def _producer(ring, tag, count):
    rng = np.random.default_rng(tag)
    for i in range(count):
        p = _payload(tag, i, int(rng.integers(0, 300)))
        assert ring.put(p.tobytes(), n_episodes=1, timeout=30.0)


def test_ring_many_producers_one_consumer():
    ctx = mp.get_context("spawn")
    ring = ShmRing(8192, lock=ctx.Lock())
    procs = [ctx.Process(target=_producer, args=(ring, t, 150)) for t in (1, 2, 3)]
    try:
        for p in procs:
            p.start()
        seen = {1: 0, 2: 0, 3: 0}
        for _ in range(450):
            m = ring.get(timeout=60.0)
            assert m is not None
            a = np.frombuffer(m[0], np.uint32)
            tag, i, n = int(a[0]), int(a[1]), int(a[2])
            assert i == seen[tag], "per-producer order"
            np.testing.assert_array_equal(a, _payload(tag, i, n))
            seen[tag] += 1
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert ring.pending_messages == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
        ring.close()


def _harvest_like(seed, n_eps):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 120, n_eps)
    hdr = np.zeros((n_eps, 16), np.uint32)
    hdr[:, 0] = rng.integers(0, 4096, n_eps)
    hdr[:, 3] = lens
    rec = rng.integers(0, 2**32, (int(lens.sum()), 12), dtype=np.uint32)
    return hdr, rec


def _queue_worker(q, seed):
    for k in range(5):
        assert q.put_records(*_harvest_like(seed * 10 + k, 40), timeout=30.0)


def test_experience_queue_records_across_processes():
    ctx = mp.get_context("spawn")
    q = ExperienceQueue(capacity_mb=1, ctx=ctx)
    procs = [ctx.Process(target=_queue_worker, args=(q, s)) for s in (1, 2)]
    try:
        for p in procs:
            p.start()
        got = []
        for _ in range(10):
            m = q.get_records(timeout=60.0)
            assert m is not None
            got.append(m)
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        expect = {}
        for s in (1, 2):
            for k in range(5):
                h, r = _harvest_like(s * 10 + k, 40)
                expect[h.tobytes()] = r
        for h, r in got:
            np.testing.assert_array_equal(expect.pop(h.tobytes()), r)
        assert not expect
        assert q.qsize() == 0
        with pytest.raises(queue.Empty):
            q.get(timeout=0.05)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
        q.close()


def test_message_pack_round_trip():
    h, r = _harvest_like(7, 13)
    h2, r2 = unpack_message(pack_message(h, r))
    np.testing.assert_array_equal(h, h2)
    np.testing.assert_array_equal(r, r2)
    h0, r0 = unpack_message(pack_message(np.zeros((0, 16), np.uint32), np.zeros((0, 12), np.uint32)))
    assert h0.shape == (0, 16) and r0.shape == (0, 12)


def test_queue_side_imports_without_torch():
    """The CPU-side queue (multi.experience_queue, bgx.records) loads neither
    torch nor libbgx.so: the package re-exports are lazy (PEP 562), while
    `from multi import ParameterManager, Worker, ExperienceQueue,
    worker_function` (main.py:2) still resolves."""
    import subprocess
    import sys
    from conftest import PKG
    code = ("import sys; sys.path.insert(0, %r); import multi.experience_queue, bgx.records; "
            "print('torch' in sys.modules, 'bgx._lib' in sys.modules)" % PKG)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True).stdout
    assert out.split() == ["False", "False"]
    code = ("import sys; sys.path.insert(0, %r); "
            "from multi import ParameterManager, Worker, ExperienceQueue, worker_function; print('ok')" % PKG)
    assert subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          check=True).stdout.strip() == "ok"
