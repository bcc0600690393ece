"""A restatement of the reference trainer process's self-play plumbing
(src/main.py:65-91 and 117-133), without the trainer: a
multiprocessing.Manager lock / Value / dict behind ParameterManager, an
ExperienceQueue, worker processes started with Process(target=
worker_function, args=(i, parameter_manager, experience_queue)), and the
`experience_queue.get(timeout=1)` loop with queue.Empty handling, each
Episode converted with `episode.to_tensor(device=...)` as main.py:129-130
does before Trainer.update. Imports `multi` / `environments` from whatever
sys.path resolves first -- the build's packages under the drop-in.
Test infrastructure (the reference itself is not on the GPU box)."""
import multiprocessing
import queue
import time


def run(n_episodes, n_workers=1, device="cuda", timeout_s=240.0):
    from multi import ExperienceQueue, ParameterManager, worker_function   # main.py:2

    ctx = multiprocessing.get_context("spawn")   # main.py:164-167
    manager = ctx.Manager()                      # main.py:65-73
    lock = manager.Lock()
    version = manager.Value("i", 1)
    parameters = manager.dict()
    parameter_manager = ParameterManager(lock, version, parameters)
    experience_queue = ExperienceQueue(ctx=ctx)  # main.py:82
    procs = []
    for i in range(n_workers):                   # main.py:85-91
        p = ctx.Process(target=worker_function, args=(i, parameter_manager, experience_queue))
        p.start()
        procs.append(p)
    episodes, empties = [], 0
    t0 = time.monotonic()
    try:
        while len(episodes) < n_episodes:        # main.py:115-137
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError(f"{len(episodes)} episodes after {timeout_s} s")
            try:
                episode = experience_queue.get(timeout=1)
                episodes.append(episode)
            except queue.Empty:
                empties += 1
        state_dict = parameter_manager.get_parameters()   # main.py:105
        for episode in episodes:                 # main.py:129-130
            episode.to_tensor(device=device)
    finally:
        for p in procs:                          # main.py:159-161
            p.terminate()
            p.join(timeout=30)
        experience_queue.close()
        manager.shutdown()
    return episodes, state_dict, empties
