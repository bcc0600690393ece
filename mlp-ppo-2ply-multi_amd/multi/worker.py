"""Worker / worker_function (src/multi/worker.py:17-179) on MI355X lanes.

The reference spawns 7 CPU processes (src/main.py:86-91), each playing one
game at a time. Here worker `worker_id` drives one bgx.Engine per GPU it is
given (gpus_for_worker: GPU g goes to worker g mod 7, so the reference's
hard-coded 7 workers cover all 8 GPUs of a node — worker 0 drives GPUs 0 and 7;
workers without a GPU return immediately), stepping thousands of lanes per
GPU and putting every finished Episode on the queue exactly as
play_episode/run do (worker.py:47-76). Each cycle queues the next launch and
its harvest before the host reads the previous harvest (harvest_enqueue /
harvest_fetch), so the GPUs keep stepping while the host copies and queues.
Parameters are re-read when the version advances (worker.py:66-76), at the
start of every cycle, before its launch is queued: a new version steers the
very next launch (set_weights waits for the launch in flight, so an update
costs one pipeline drain, and only when the version moved).

Knobs (environment): BGX_WORKERS (7: main.py:86's worker count),
BGX_GPU_MAP (explicit GPUs per worker id: "0;1;2;3;4;5;6,7" = worker 6 drives
GPUs 6 and 7), BGX_LANES (4096 per GPU), BGX_PLY (1), BGX_K_TOP (4),
BGX_BALANCE (1: balanced fused launches, include/bgx.h bgx_config.balance),
BGX_STEPS_PER_HARVEST (100), BGX_MAX_PENDING (2000 episodes queued before the
engine pauses: the queue's Python consumer is far slower than the engine),
BGX_BULK (1: one shared-memory message per harvest through
ExperienceQueue.put_records; 0: one pickled Episode per put, as the reference).
"""
import os
import time

import numpy as np
import torch

from bgx import Engine
from bgx.episodes import to_episodes
from environments import Episode, Experience, Player


def _env_int(name, default):
    return int(os.environ.get(name, default))


def gpus_for_worker(worker_id, n_gpu, n_workers=7, gpu_map=None):
    """GPUs worker `worker_id` drives. gpu_map ("0;1;2;3;4;5;6,7": worker ids
    separated by ';', GPUs by ','), else GPU g -> worker g mod n_workers, so
    main.py's 7 workers (main.py:86) cover every GPU of an 8-GPU node."""
    if gpu_map:
        per = [p.strip() for p in gpu_map.split(";")]
        if worker_id >= len(per) or not per[worker_id]:
            return []
        gpus = [int(x) for x in per[worker_id].split(",") if x.strip()]
        bad = [g for g in gpus if not 0 <= g < n_gpu]
        if bad:
            raise ValueError(f"BGX_GPU_MAP names GPU(s) {bad}; {n_gpu} visible")
        return gpus
    return [g for g in range(n_gpu) if g % max(1, n_workers) == worker_id]


class Worker:
    def __init__(self, worker_id, parameter_manager, experience_queue):
        self.worker_id = worker_id
        self.parameter_manager = parameter_manager
        self.experience_queue = experience_queue
        self.temperature = self.parameter_manager.get_temperature()
        self.state_dict = self.parameter_manager.get_parameters()
        self.current_version = self.parameter_manager.get_version()
        n_gpu = torch.cuda.device_count()
        self.devices = gpus_for_worker(worker_id, n_gpu, _env_int("BGX_WORKERS", 7), os.environ.get("BGX_GPU_MAP"))
        self.device = self.devices[0] if self.devices else None
        self.lanes = _env_int("BGX_LANES", 4096)
        self.balance = _env_int("BGX_BALANCE", 1) != 0
        self.ply = _env_int("BGX_PLY", 1)
        self.k_top = _env_int("BGX_K_TOP", 4)
        self.steps_per_harvest = _env_int("BGX_STEPS_PER_HARVEST", 100)
        self.max_pending = _env_int("BGX_MAX_PENDING", 2000)
        self.engines = []
        self.engine = None   # the first GPU's engine
        self._staging = []   # per engine: page-locked host buffer for DMA-engine harvest copies
        self._pending = []   # the engines' harvest tickets of the launch in flight

    def _ensure_engine(self):
        """One engine per GPU of this worker: global lanes [g * lanes, (g + 1) *
        lanes) on GPU g, seeded per GPU (the lanes of GPU g are the same
        whichever worker drives it)."""
        if not self.engines:
            for g in self.devices:
                torch.cuda.set_device(g)
                e = Engine(lanes=self.lanes, seed=1000003 * (g + 1), ply=self.ply, k_top=self.k_top,
                           lane_base=g * self.lanes, balance=self.balance)
                e.set_weights(self.state_dict, self.temperature, self.current_version)
                self.engines.append(e)
            torch.cuda.set_device(self.devices[0])
            self.engine = self.engines[0]
        return self.engines

    def _maybe_update(self):
        new_version = self.parameter_manager.get_version()
        if new_version > self.current_version:
            self.state_dict = self.parameter_manager.get_parameters()
            self.temperature = self.parameter_manager.get_temperature()
            for e in self.engines:
                e.set_weights(self.state_dict, self.temperature, new_version)
            self.current_version = new_version

    def _step_all(self, steps):
        """One pipelined cycle over this worker's engines: every engine's next
        launch and its harvest ticket are queued first (the GPUs step
        concurrently), then the PREVIOUS cycle's tickets are fetched, so the
        host decodes / copies a harvest while the next launch runs and an
        engine never waits for the host between launches (the reference's loop,
        worker.py:47-76, plays one episode at a time). The harvests returned
        are views into the engines' buffers, valid until the next cycle
        queues its tickets; the first cycle returns none."""
        engines = self._ensure_engine()
        self._maybe_update()   # before the launch is queued: no launch runs on stale weights
        tickets = []
        for e in engines:
            with torch.cuda.device(e.device):
                e.step(steps or self.steps_per_harvest)
                tickets.append(e.harvest_enqueue())
        harvests = []
        for e, t in zip(engines, self._pending):
            with torch.cuda.device(e.device):
                harvests.append(e.harvest_fetch(t))
        self._pending = tickets
        return harvests

    def play_episodes(self, steps=None):
        """Advance all lanes one launch and return the Episodes of the previous
        launch's harvest (already to_numpy()'d)."""
        out = []
        for e, h in zip(self.engines, self._step_all(steps)):
            # on the harvest's own device: its decode kernels and the .cpu() that
            # follows use that device's current stream
            with torch.cuda.device(e.device):
                out += to_episodes(h, Episode, Experience, Player)
        return out

    def harvest_records(self, steps=None):
        """Advance all lanes one launch; return the previous launch's finished
        episodes as compact host arrays (headers uint32 [n, 16], records
        uint32 [m, 12]) for the bulk queue path (each episode's records
        contiguous, in header order, GPU by GPU). With one GPU they are views
        into the DMA staging buffer, valid until the next call."""
        hs = self._step_all(steps)
        # device -> host on the DMA engines (bgx/hostcopy.py): a torch copy here
        # is a blit kernel that would wait for the launch just queued, idling the
        # GPU for the host's work every cycle
        if not self._staging:
            from bgx.hostcopy import Staging
            self._staging = [Staging(e.device.index) for e in self.engines]
        parts = [st.copy(h) for st, h in zip(self._staging, hs)]
        hdr = [p[0] for p in parts]
        rec = [p[1] for p in parts]
        if not hs:
            return np.zeros((0, 16), np.uint32), np.zeros((0, 12), np.uint32)
        if len(hs) == 1:
            return hdr[0], rec[0]
        return np.concatenate(hdr), np.concatenate(rec)

    def run(self):
        if self.device is None:
            print(f"Worker {self.worker_id}: no GPU for this worker id; idle.")
            return
        print(f"Worker {self.worker_id} starting on cuda:{self.devices} with {self.lanes} lanes per GPU.")
        bulk = hasattr(self.experience_queue, "put_records") and os.environ.get("BGX_BULK", "1") != "0"
        while True:
            if bulk:
                hdr, rec = self.harvest_records()
                if hdr.shape[0]:
                    self.experience_queue.put_records(hdr, rec)
            else:
                for episode in self.play_episodes():
                    self.experience_queue.put(episode)
            while self.experience_queue.qsize() > self.max_pending:
                time.sleep(0.01)
                self._maybe_update()


def worker_function(worker_id, parameter_manager, experience_queue):
    worker = Worker(worker_id, parameter_manager, experience_queue)
    worker.run()
