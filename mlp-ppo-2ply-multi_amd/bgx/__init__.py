"""bgx — MI355X-native backgammon self-play engine (libbgx.so + thin Python host).

Public surface:
  bgx.ops      movegen / encode / pack / unpack / Net (stateless parity entry points)
  bgx.Engine   lanes of self-play on one device (bgx_engine_* in include/bgx.h)
  bgx.episodes harvested records -> reference-shaped Episode / Experience objects
  bgx.dist     one-process-per-GPU sharding, RCCL episode gather / weight broadcast
  bgx.records  the harvest wire format (numpy only)

The re-exports below load on first use (PEP 562), so `import bgx.records`
(the CPU-side queue's wire format) pulls in neither torch nor libbgx.so.
"""
import importlib

_EXPORTS = {
    "BgxError": "._lib", "LIB_PATH": "._lib", "lib": "._lib",
    "Engine": ".engine", "Harvest": ".engine",
    "BackgammonPolicyNetwork": ".net",
}
_SUBMODULES = ("ops", "dist", "episodes", "records", "trainer", "net", "engine")

__all__ = list(_EXPORTS) + ["ops"]


def __getattr__(name):
    if name in _EXPORTS:
        return getattr(importlib.import_module(_EXPORTS[name], __name__), name)
    if name in _SUBMODULES:
        return importlib.import_module("." + name, __name__)
    raise AttributeError(f"module 'bgx' has no attribute {name!r}")
