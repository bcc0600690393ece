"""ctypes wrapper over the CPU oracle ``libbgref.so``.

ORACLE — TEST INFRASTRUCTURE ONLY. Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import this module; the product
path (``libbgx.so`` and the ``bgx`` package) never does. Each wrapped function
restates the reference file:line cited in ``bgref.h`` / ``bgref.c`` and is
pinned by ``tests/test_oracle_golden.py`` against the golden vectors that
``tools/gen_golden.py`` produced by importing the reference in the build
container.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libbgref.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
f32p = ctypes.POINTER(ctypes.c_float)
f64p = ctypes.POINTER(ctypes.c_double)


class Env(ctypes.Structure):
    _fields_ = [
        ("board", ctypes.c_uint8 * 52),
        ("current_player", ctypes.c_int),
        ("game_over", ctypes.c_int),
        ("roll", ctypes.c_int * 2),
        ("close_out_given", ctypes.c_int * 2),
        ("prime_given", ctypes.c_int * 2),
        ("num_moves", ctypes.c_int),
        ("full_moves", ctypes.c_int),
        ("max_legal_moves", ctypes.c_int),
        ("legal_boards", u8p),
        ("dice", ctypes.POINTER(ctypes.c_int)),
        ("n_dice", ctypes.c_int),
        ("dice_pos", ctypes.c_int),
    ]


class StepResult(ctypes.Structure):
    _fields_ = [
        ("reward", ctypes.c_float),
        ("done", ctypes.c_int),
        ("info_current_player", ctypes.c_int),
        ("winner", ctypes.c_int),
        ("win_type", ctypes.c_int),
        ("close_out_reward", ctypes.c_int),
        ("prime_reward", ctypes.c_int),
        ("kind", ctypes.c_int),
    ]


def build() -> str:
    """Compile libbgref.so with the committed Makefile (gcc only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "bgref.c")
        ):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.bgref_movegen_full.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p,
                                         ctypes.c_int, u8p, u8p]
        L.bgref_movegen_full.restype = ctypes.c_int
        L.bgref_encode.argtypes = [u8p, ctypes.c_int, ctypes.c_int, f32p]
        L.bgref_value.argtypes = [f32p, f32p, f32p, f32p, f32p, ctypes.c_int, f64p]
        L.bgref_value_f32.argtypes = [f32p, f32p, f32p, f32p, f32p, ctypes.c_int, f32p]
        for name in ("bgref_check_game_over", "bgref_check_for_gammon",
                     "bgref_check_for_backgammon", "bgref_made_at_least_five_prime",
                     "bgref_is_closed_out"):
            getattr(L, name).argtypes = [u8p, ctypes.c_int]
            getattr(L, name).restype = ctypes.c_int
        L.bgref_two_ply_response.argtypes = [u8p, ctypes.c_int, f32p, f32p, f32p, f32p]
        L.bgref_two_ply_response.restype = ctypes.c_double
        L.bgref_env_init.argtypes = [ctypes.POINTER(Env), u8p, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int), ctypes.c_int]
        L.bgref_env_reset.argtypes = [ctypes.POINTER(Env)]
        L.bgref_env_step.argtypes = [ctypes.POINTER(Env), ctypes.c_int,
                                     ctypes.POINTER(StepResult)]
        L.bgref_philox4x32.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.POINTER(ctypes.c_uint32)]
        L.bgref_selfplay_bench.argtypes = [f32p, f32p, f32p, f32p, ctypes.c_float,
                                           ctypes.c_uint64, ctypes.c_int, ctypes.c_double,
                                           ctypes.POINTER(ctypes.c_longlong),
                                           ctypes.POINTER(ctypes.c_longlong), f64p]
        L.bgref_selfplay_bench.restype = ctypes.c_longlong
        L.bgref_selfplay_bench_ply.argtypes = [f32p, f32p, f32p, f32p, ctypes.c_float,
                                               ctypes.c_uint64, ctypes.c_int, ctypes.c_double,
                                               ctypes.c_int, ctypes.POINTER(ctypes.c_longlong),
                                               ctypes.POINTER(ctypes.c_longlong), f64p]
        L.bgref_selfplay_bench_ply.restype = ctypes.c_longlong
        L.bgref_selfplay_bench_warm.argtypes = [f32p, f32p, f32p, f32p, ctypes.c_float,
                                                ctypes.c_uint64, ctypes.c_int, ctypes.c_double,
                                                ctypes.c_int, ctypes.c_longlong,
                                                ctypes.POINTER(ctypes.c_longlong),
                                                ctypes.POINTER(ctypes.c_longlong), f64p]
        L.bgref_selfplay_bench_warm.restype = ctypes.c_longlong
        _lib = L
    return _lib


def _u8(a):
    return a.ctypes.data_as(u8p)


def _f32(a):
    return a.ctypes.data_as(f32p)


def movegen(board, player, d0, d1, cap=8192, with_sub=False):
    """Ordered result boards of get_all_possible_moves (uint8 [n, 52]), nsub [n]."""
    board = np.ascontiguousarray(board, dtype=np.uint8)
    out = np.zeros((cap, 52), np.uint8)
    nsub = np.zeros(cap, np.uint8)
    sub = np.zeros((cap, 4, 3), np.uint8) if with_sub else None
    n = lib().bgref_movegen_full(_u8(board), int(player), int(d0), int(d1), _u8(out), cap,
                                 _u8(nsub), _u8(sub) if with_sub else None)
    w = min(n, cap)
    if with_sub:
        return n, out[:w], nsub[:w], sub[:w]
    return n, out[:w], nsub[:w]


def encode(board, player, layout=0):
    board = np.ascontiguousarray(board, dtype=np.uint8)
    out = np.zeros(198, np.float32)
    lib().bgref_encode(_u8(board), int(player), int(layout), _f32(out))
    return out


def encode_many(boards, players, layout=0):
    boards = np.ascontiguousarray(boards, dtype=np.uint8).reshape(-1, 52)
    players = np.broadcast_to(np.asarray(players), (boards.shape[0],))
    return np.stack([encode(b, p, layout) for b, p in zip(boards, players)]) if len(boards) \
        else np.zeros((0, 198), np.float32)


def value(weights, x):
    """V in float64 for x float32 [n, 198]; weights dict W1,b1,w2,b2 (fp32)."""
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1, 198)
    W1, b1, w2, b2 = (np.ascontiguousarray(weights[k], dtype=np.float32)
                      for k in ("W1", "b1", "w2", "b2"))
    out = np.zeros(x.shape[0], np.float64)
    lib().bgref_value(_f32(W1), _f32(b1), _f32(w2), _f32(b2), _f32(x), x.shape[0],
                      out.ctypes.data_as(f64p))
    return out


def predicate(name, board, player):
    board = np.ascontiguousarray(board, dtype=np.uint8)
    return bool(getattr(lib(), "bgref_" + name)(_u8(board), int(player)))


def two_ply_response(weights, board, opponent):
    board = np.ascontiguousarray(board, dtype=np.uint8)
    W1, b1, w2, b2 = (np.ascontiguousarray(weights[k], dtype=np.float32)
                      for k in ("W1", "b1", "w2", "b2"))
    return lib().bgref_two_ply_response(_u8(board), int(opponent), _f32(W1), _f32(b1),
                                        _f32(w2), _f32(b2))


class OracleEnv:
    """BackgammonEnv (src/environments/backgammon_env.py) driven by a recorded
    sequence of single-die draws."""

    def __init__(self, dice, max_legal_moves=500):
        self._dice = (ctypes.c_int * max(1, len(dice)))(*[int(d) for d in dice])
        self._legal = np.zeros((max_legal_moves, 52), np.uint8)
        self.env = Env()
        lib().bgref_env_init(ctypes.byref(self.env), _u8(self._legal), max_legal_moves,
                             self._dice, len(dice))

    def reset(self):
        if lib().bgref_env_reset(ctypes.byref(self.env)) != 0:
            raise RuntimeError("dice exhausted")

    def step(self, action):
        r = StepResult()
        if lib().bgref_env_step(ctypes.byref(self.env), int(action), ctypes.byref(r)) != 0:
            raise RuntimeError("dice exhausted")
        return r

    @property
    def board(self):
        return np.frombuffer(bytes(self.env.board), np.uint8).copy()

    @property
    def legal_boards(self):
        return self._legal[: self.env.num_moves].copy()


def philox(key, ctr_hi, ctr_lo):
    out = (ctypes.c_uint32 * 4)()
    lib().bgref_philox4x32(key, ctr_hi, ctr_lo, out)
    return list(out)


def selfplay_bench(weights, temperature=1.5, seed=0, n_threads=1, seconds=5.0, ply=1, warmup=0):
    W1, b1, w2, b2 = (np.ascontiguousarray(weights[k], dtype=np.float32)
                      for k in ("W1", "b1", "w2", "b2"))
    dec = ctypes.c_longlong(0)
    eps = ctypes.c_longlong(0)
    el = ctypes.c_double(0)
    steps = lib().bgref_selfplay_bench_warm(_f32(W1), _f32(b1), _f32(w2), _f32(b2),
                                            float(temperature), int(seed), int(n_threads),
                                            float(seconds), int(ply), int(warmup), ctypes.byref(dec),
                                            ctypes.byref(eps), ctypes.byref(el))
    return {"steps": int(steps), "decisions": int(dec.value), "episodes": int(eps.value),
            "elapsed": float(el.value), "threads": int(n_threads)}
