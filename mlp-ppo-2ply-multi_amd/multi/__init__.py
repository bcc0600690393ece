"""Drop-in for the reference's src/multi package (src/multi/__init__.py:1-5):
`from multi import ParameterManager, Worker, ExperienceQueue, worker_function`
keeps working under src/main.py, with self-play running on MI355X lanes."""
from .experience_queue import ExperienceQueue
from .parameter_manager import ParameterManager
from .worker import Worker, worker_function

__all__ = ["ExperienceQueue", "ParameterManager", "Worker", "worker_function"]
