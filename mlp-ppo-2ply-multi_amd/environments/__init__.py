"""Drop-in for the reference's src/environments Episode/Experience containers
(src/environments/__init__.py:1-3). BackgammonEnv itself is replaced by the
GPU lanes of bgx.Engine (see multi.worker)."""
from .episode import Episode, Experience, Player

__all__ = ["Episode", "Experience", "Player"]
