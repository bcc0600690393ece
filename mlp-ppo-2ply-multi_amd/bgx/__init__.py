"""bgx — MI355X-native backgammon self-play engine (libbgx.so + thin Python host).

Public surface:
  bgx.ops      movegen / encode / pack / unpack / Net (stateless parity entry points)
  bgx.Engine   lanes of self-play on one device (bgx_engine_* in include/bgx.h)
  bgx.episodes harvested records -> reference-shaped Episode / Experience objects
  bgx.dist     one-process-per-GPU sharding, RCCL episode gather / weight broadcast
"""
from ._lib import BgxError, LIB_PATH, lib
from .engine import Engine, Harvest
from .net import BackgammonPolicyNetwork
from . import ops

__all__ = ["BgxError", "LIB_PATH", "lib", "Engine", "Harvest", "BackgammonPolicyNetwork", "ops"]
