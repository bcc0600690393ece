"""ExperienceQueue (src/multi/experience_queue.py:5-13): a multiprocessing queue of Episodes."""
from multiprocessing import Queue


class ExperienceQueue:
    def __init__(self):
        self.queue = Queue()

    def put(self, episode):
        self.queue.put(episode)

    def get(self, timeout=None):
        return self.queue.get(timeout=timeout)

    def qsize(self):
        try:
            return self.queue.qsize()
        except NotImplementedError:   # macOS
            return 0
