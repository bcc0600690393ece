"""ctypes binding of libbgx.so (include/bgx.h).

torch is imported first on purpose: torch-ROCm carries its own
libamdhip64.so.7; loading it before libbgx.so makes the dynamic loader bind
libbgx.so to that same HIP runtime (matching SONAME), so torch's device
pointers and streams are valid inside the library.

There is no fallback: if libbgx.so is missing or was built for another
target, every op raises. Build it with ``make -C mlp-ppo-2ply-multi_amd/csrc``
(or ``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load; see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BGX_LIB", os.path.join(_HERE, "libbgx.so"))

c_int, c_float, c_double, c_u64, c_void_p = (ctypes.c_int, ctypes.c_float, ctypes.c_double,
                                             ctypes.c_uint64, ctypes.c_void_p)

ABI_VERSION = 10


class BgxError(RuntimeError):
    """A libbgx call returned an error code (message from bgx_last_error)."""


class Config(ctypes.Structure):
    _fields_ = [
        ("lanes", c_int), ("lane_base", c_int), ("seed", c_u64), ("ply", c_int), ("k_top", c_int),
        ("alpha", c_float), ("beta", c_float), ("max_steps", c_int), ("max_legal", c_int),
        ("ring", c_int), ("ep_cap", c_int), ("cand_per_lane", c_int), ("reply_per_lane", c_int),
        ("greedy", c_int), ("fused", c_int), ("reply_sample", c_int), ("balance", c_int),
    ]


class HarvestInfo(ctypes.Structure):
    _fields_ = [("n_episodes", c_int), ("n_records", c_int), ("d_headers", c_void_p),
                ("d_records", c_void_p)]


class Stats(ctypes.Structure):
    _fields_ = [("env_steps", c_u64), ("decisions", c_u64), ("episodes", c_u64),
                ("value_rows", c_u64), ("movegen_jobs", c_u64), ("fallback_jobs", c_u64), ("gap_rows", c_u64)]


# every entry point declared in include/bgx.h: name -> (restype, argtypes)
SIGNATURES = {
    "bgx_abi_version": (c_int, []),
    "bgx_last_error": (ctypes.c_char_p, []),
    "bgx_check_boards": (c_int, [c_void_p, c_void_p, c_void_p, c_int, ctypes.POINTER(ctypes.c_uint32),
                                 ctypes.POINTER(ctypes.c_int32), c_void_p]),
    "bgx_check_boards_host": (c_int, [c_void_p, c_void_p, c_void_p, c_int, ctypes.POINTER(ctypes.c_uint32),
                                      ctypes.POINTER(ctypes.c_int32)]),
    "bgx_movegen": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "bgx_encode": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "bgx_encode_packed": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "bgx_net_create": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, ctypes.POINTER(c_void_p)]),
    "bgx_net_destroy": (c_int, [c_void_p]),
    "bgx_value": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "bgx_value_boards": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "bgx_two_ply": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "bgx_two_ply_sampled": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_u64, c_void_p, c_void_p]),
    "bgx_config_default": (None, [ctypes.POINTER(Config)]),
    "bgx_engine_create": (c_int, [c_int, ctypes.POINTER(Config), ctypes.POINTER(c_void_p)]),
    "bgx_engine_destroy": (c_int, [c_void_p]),
    "bgx_set_weights": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_u64]),
    "bgx_engine_set_dice": (c_int, [c_void_p, c_void_p, c_int]),
    "bgx_step": (c_int, [c_void_p, c_int, c_void_p]),
    "bgx_sync": (c_int, [c_void_p]),
    "bgx_harvest": (c_int, [c_void_p, ctypes.POINTER(HarvestInfo), c_void_p]),
    "bgx_harvest_enqueue": (c_int, [c_void_p, ctypes.POINTER(c_int), c_void_p]),
    "bgx_harvest_fetch": (c_int, [c_void_p, c_int, ctypes.POINTER(HarvestInfo)]),
    "bgx_get_stats": (c_int, [c_void_p, ctypes.POINTER(Stats)]),
    "bgx_engine_peek": (c_int, [c_void_p, c_int, c_void_p, c_u64, ctypes.POINTER(c_u64)]),
    "bgx_set_timing": (c_int, [c_void_p, c_int]),
    "bgx_get_timing": (c_int, [c_void_p, ctypes.POINTER(c_double), ctypes.POINTER(c_int),
                               ctypes.POINTER(c_double), ctypes.POINTER(c_int)]),
    "bgx_td0_update": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                               c_float, c_float, c_void_p, c_void_p]),
    "bgx_host_register": (c_int, [c_void_p, c_u64]),
    "bgx_host_unregister": (c_int, [c_void_p]),
    "bgx_copy_async": (c_int, [c_void_p, c_void_p, c_u64, c_int, c_void_p]),
    "bgx_dma_copy_d2h": (c_int, [c_void_p, c_void_p, c_u64, c_int, ctypes.POINTER(c_u64)]),
    "bgx_dma_wait": (c_int, [c_u64, c_int]),
    "bgx_dma_copy_d2d": (c_int, [c_void_p, c_int, c_void_p, c_int, c_u64, ctypes.POINTER(c_u64)]),
    "bgx_ipc_export": (c_int, [c_void_p, c_void_p, ctypes.POINTER(c_u64)]),
    "bgx_ipc_open": (c_int, [c_void_p, c_u64, ctypes.POINTER(c_void_p)]),
    "bgx_ipc_close": (c_int, [c_void_p, c_u64]),
    "bgx_reply_moves": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "bgx_pack": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "bgx_unpack": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
}

_lib = None


def lib():
    """The loaded libbgx.so (raises if it is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BgxError(f"libbgx.so not found at {LIB_PATH}; build it with "
                           f"`make -C mlp-ppo-2ply-multi_amd/csrc` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.bgx_abi_version() != ABI_VERSION:
            raise BgxError(f"libbgx ABI {L.bgx_abi_version()} != expected {ABI_VERSION}")
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().bgx_last_error().decode(errors="replace")
        raise BgxError(f"{what or 'libbgx'} failed ({rc}): {msg}")


def stream_handle(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def require_cuda(*tensors) -> None:
    if not torch.cuda.is_available():
        raise BgxError("bgx ops need an MI355X (torch.cuda.is_available() is False); "
                       "there is no CPU fallback")
    for t in tensors:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise BgxError("bgx ops take contiguous device tensors")
