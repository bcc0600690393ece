"""Worker / worker_function (src/multi/worker.py:17-179) on MI355X lanes.

The reference spawns 7 CPU processes (src/main.py:86-91), each playing one
game at a time. Here worker `worker_id` drives one bgx.Engine on GPU
`worker_id` (ids beyond the visible GPU count return immediately, so the
reference's hard-coded 7 workers map onto the node's GPUs), stepping
thousands of lanes and putting every finished Episode on the queue exactly as
play_episode/run do (worker.py:47-76). Parameters are re-read when the
version advances (worker.py:66-76), at every harvest.

Knobs (environment): BGX_LANES (4096), BGX_PLY (1), BGX_K_TOP (4),
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


class Worker:
    def __init__(self, worker_id, parameter_manager, experience_queue):
        self.worker_id = worker_id
        self.parameter_manager = parameter_manager
        self.experience_queue = experience_queue
        self.temperature = self.parameter_manager.get_temperature()
        self.state_dict = self.parameter_manager.get_parameters()
        self.current_version = self.parameter_manager.get_version()
        n_gpu = torch.cuda.device_count()
        self.device = worker_id if worker_id < n_gpu else None
        self.lanes = _env_int("BGX_LANES", 4096)
        self.ply = _env_int("BGX_PLY", 1)
        self.k_top = _env_int("BGX_K_TOP", 4)
        self.steps_per_harvest = _env_int("BGX_STEPS_PER_HARVEST", 100)
        self.max_pending = _env_int("BGX_MAX_PENDING", 2000)
        self.engine = None

    def _ensure_engine(self):
        if self.engine is None:
            torch.cuda.set_device(self.device)
            self.engine = Engine(lanes=self.lanes, seed=1000003 * (self.worker_id + 1), ply=self.ply,
                                 k_top=self.k_top, lane_base=self.worker_id * self.lanes)
            self.engine.set_weights(self.state_dict, self.temperature, self.current_version)
        return self.engine

    def _maybe_update(self):
        new_version = self.parameter_manager.get_version()
        if new_version > self.current_version:
            self.state_dict = self.parameter_manager.get_parameters()
            self.temperature = self.parameter_manager.get_temperature()
            self.engine.set_weights(self.state_dict, self.temperature, new_version)
            self.current_version = new_version

    def play_episodes(self, steps=None):
        """Advance all lanes and return the Episodes that finished (already to_numpy()'d)."""
        eng = self._ensure_engine()
        eng.step(steps or self.steps_per_harvest)
        return to_episodes(eng.harvest(), Episode, Experience, Player)

    def harvest_records(self, steps=None):
        """Advance all lanes; return the finished episodes as compact host arrays
        (headers uint32 [n, 16], records uint32 [m, 12]) for the bulk queue path."""
        eng = self._ensure_engine()
        eng.step(steps or self.steps_per_harvest)
        h = eng.harvest()
        return (h.headers.cpu().numpy().view(np.uint32), h.records.cpu().numpy().view(np.uint32))

    def run(self):
        if self.device is None:
            print(f"Worker {self.worker_id}: no GPU for this worker id; idle.")
            return
        print(f"Worker {self.worker_id} starting on cuda:{self.device} with {self.lanes} lanes.")
        bulk = hasattr(self.experience_queue, "put_records") and os.environ.get("BGX_BULK", "1") != "0"
        while True:
            if bulk:
                self.experience_queue.put_records(*self.harvest_records())
            else:
                for episode in self.play_episodes():
                    self.experience_queue.put(episode)
            self._maybe_update()
            while self.experience_queue.qsize() > self.max_pending:
                time.sleep(0.01)
                self._maybe_update()


def worker_function(worker_id, parameter_manager, experience_queue):
    worker = Worker(worker_id, parameter_manager, experience_queue)
    worker.run()
