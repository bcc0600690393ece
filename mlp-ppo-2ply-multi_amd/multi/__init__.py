"""Drop-in for the reference's src/multi package (src/multi/__init__.py:1-5):
`from multi import ParameterManager, Worker, ExperienceQueue, worker_function`
keeps working under src/main.py, with self-play running on MI355X lanes.

The names load on first use (PEP 562): a process that only needs the queue
(`multi.experience_queue`, numpy + the shared-memory ring) imports neither
torch nor the engine."""
import importlib

_EXPORTS = {"ExperienceQueue": ".experience_queue", "ParameterManager": ".parameter_manager",
            "Worker": ".worker", "worker_function": ".worker"}

__all__ = list(_EXPORTS)


def __getattr__(name):
    if name in _EXPORTS:
        return getattr(importlib.import_module(_EXPORTS[name], __name__), name)
    raise AttributeError(f"module 'multi' has no attribute {name!r}")
