"""Stateless device ops over libbgx.so (the parity entry points of include/bgx.h).

Each op mirrors one reference function on a batch of boards:
  movegen      get_all_possible_moves + execute_full_move_on_board_copy
               (backgammon/moves/generate_all_moves.py:7-90, environments/env_helper.py:27-91)
  encode       ImmutableBoard.get_board_features (board/immutable_board.py:86-128),
               layout=1: generate_board_tensor.compute_features (:98-140)
  Net.value    BackgammonPolicyNetwork.forward (agents/policy_network.py:53-70)
Boards are uint8 [n, 52] device tensors in the reference's field order.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._lib import check, lib, ptr, require_cuda, stream_handle


def _u8(t, shape_last=None):
    t = torch.as_tensor(t)
    if t.dtype != torch.uint8:
        t = t.to(torch.uint8)
    if not t.is_cuda:
        t = t.cuda()
    return t.contiguous()


def movegen(boards, player, dice, cap: int = 512, stream=None):
    """Ordered result boards for n (board, player, dice) jobs.

    Returns (out uint8 [n, cap, 52], count int32 [n]); count is the full
    number of results, rows k >= min(count, cap) are unspecified."""
    boards, player, dice = _u8(boards).view(-1, 52), _u8(player).view(-1), _u8(dice).view(-1, 2)
    n = boards.shape[0]
    require_cuda(boards, player, dice)
    out = torch.empty((n, cap, 52), dtype=torch.uint8, device=boards.device)
    cnt = torch.empty((n,), dtype=torch.int32, device=boards.device)
    check(lib().bgx_movegen(ptr(boards), ptr(player), ptr(dice), n, ptr(out), ptr(cnt), cap,
                            stream_handle(stream)), "bgx_movegen")
    return out, cnt


BAD_BITS = {1: "a point held by both players", 2: "more than 15 checkers of a player",
            4: "a count above 15", 8: "a die outside 1..6", 16: "a player not 0/1"}


def check_boards(boards, player=None, dice=None, stream=None):
    """The input-domain check of the stateless ops (include/bgx.h BGX_BADF_*)
    on the device: returns (flags, first bad index or -1)."""
    boards = _u8(boards).view(-1, 52)
    require_cuda(boards)
    player = None if player is None else _u8(player).view(-1)
    dice = None if dice is None else _u8(dice).view(-1, 2)
    f, first = ctypes.c_uint32(0), ctypes.c_int32(-1)
    check(lib().bgx_check_boards(ptr(boards), ptr(player), ptr(dice), boards.shape[0], ctypes.byref(f),
                                 ctypes.byref(first), stream_handle(stream)), "bgx_check_boards")
    return int(f.value), int(first.value)


def encode(boards, player, layout: int = 0, stream=None):
    boards, player = _u8(boards).view(-1, 52), _u8(player).view(-1)
    require_cuda(boards, player)
    n = boards.shape[0]
    out = torch.empty((n, 198), dtype=torch.float32, device=boards.device)
    check(lib().bgx_encode(ptr(boards), ptr(player), n, ptr(out), int(layout), stream_handle(stream)),
          "bgx_encode")
    return out


def encode_packed(packed, layout: int = 0, stream=None):
    """encode() of the engine's own packed boards (int32 [n, 8]: harvest
    records / headers, the indicator in word 6): no input-domain check and no
    synchronization (bgx_encode_packed; such boards come from the engine)."""
    packed = torch.as_tensor(packed)
    if not packed.is_cuda:
        packed = packed.cuda()
    packed = packed.contiguous().view(-1, 8)
    require_cuda(packed)
    n = packed.shape[0]
    out = torch.empty((n, 198), dtype=torch.float32, device=packed.device)
    check(lib().bgx_encode_packed(ptr(packed), n, ptr(out), int(layout), stream_handle(stream)),
          "bgx_encode_packed")
    return out


def reply_moves(boards, opponent, cap: int = 0, stream=None):
    """The 2-ply reply expansion (include/bgx.h bgx_reply_moves): for each
    candidate board, the opponent's afterstates for the 21 DICE_ROLLS.
    Returns (rows int32 [cap, 8] packed, off int32 [n * 21], cnt int32 [n * 21])."""
    boards, opponent = _u8(boards).view(-1, 52), _u8(opponent).view(-1)
    require_cuda(boards, opponent)
    n = boards.shape[0]
    # records (<= 64 per (board, roll) on average, generously) + per workgroup
    # of the launch (two per CU, at most ceil(7 n / 16): bgx_launch_movegen) two
    # row chunks' worth (2 x 2,048 rows: its last chunk's tail and its waves'
    # kept remainders, each smaller than one request); running out is an error
    # (BGX_E_CAPACITY), never a silent truncation
    n_cu = torch.cuda.get_device_properties(boards.device).multi_processor_count
    cap = cap or n * 21 * 64 + min(2 * n_cu, (n * 7 + 15) // 16) * 2 * 2048 + 4096
    out = torch.empty((cap, 8), dtype=torch.int32, device=boards.device)
    off = torch.empty((n * 21,), dtype=torch.int32, device=boards.device)
    cnt = torch.empty((n * 21,), dtype=torch.int32, device=boards.device)
    check(lib().bgx_reply_moves(ptr(boards), ptr(opponent), n, ptr(out), cap, ptr(off), ptr(cnt),
                                stream_handle(stream)), "bgx_reply_moves")
    return out, off, cnt


def pack(boards, player, stream=None):
    boards, player = _u8(boards).view(-1, 52), _u8(player).view(-1)
    require_cuda(boards, player)
    n = boards.shape[0]
    out = torch.empty((n, 8), dtype=torch.int32, device=boards.device)
    check(lib().bgx_pack(ptr(boards), ptr(player), n, ptr(out), stream_handle(stream)), "bgx_pack")
    return out


def unpack(packed, stream=None):
    """Packed boards (int32 [n, 8]) -> uint8 [n, 52]; the indicator player is
    bits 16.. of word 6."""
    packed = torch.as_tensor(packed).contiguous()
    require_cuda(packed)
    n = packed.shape[0]
    out = torch.empty((n, 52), dtype=torch.uint8, device=packed.device)
    check(lib().bgx_unpack(ptr(packed), n, ptr(out), stream_handle(stream)), "bgx_unpack")
    return out


def packed_player(packed):
    return ((packed[:, 6] >> 16) & 1).to(torch.uint8)


def weights_from(obj):
    """Host fp32 (W1 [128,198], b1 [128], w2 [128], b2 [1]) from a state_dict
    (fc1.weight, fc1.bias, value_head.weight, value_head.bias) or a dict with
    keys W1, b1, w2, b2."""
    if "fc1.weight" in obj:
        W1, b1 = obj["fc1.weight"], obj["fc1.bias"]
        w2, b2 = obj["value_head.weight"], obj["value_head.bias"]
    else:
        W1, b1, w2, b2 = obj["W1"], obj["b1"], obj["w2"], obj["b2"]

    def f(x, shape):
        if isinstance(x, torch.Tensor):
            x = x.detach().float().cpu().numpy()
        return np.ascontiguousarray(np.asarray(x, dtype=np.float32).reshape(shape))

    W1 = f(W1, (128, 198))
    if W1.shape != (128, 198):
        raise ValueError("fc1.weight must be [128, 198] (BackgammonPolicyNetwork hidden_size=128)")
    return W1, f(b1, (128,)), f(w2, (128,)), f(b2, (1,))


def _fp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Net:
    """Device copy of BackgammonPolicyNetwork weights (fp32 + split-fp16 MFMA fragments)."""

    def __init__(self, weights):
        W1, b1, w2, b2 = weights_from(weights)
        if not torch.cuda.is_available():
            require_cuda()
        h = ctypes.c_void_p()
        check(lib().bgx_net_create(_fp(W1), _fp(b1), _fp(w2), _fp(b2), ctypes.byref(h)),
              "bgx_net_create")
        self._h = h
        self._destroy = lib().bgx_net_destroy   # bound now: module globals are gone at interpreter exit

    def __del__(self):
        h = getattr(self, "_h", None)
        destroy = getattr(self, "_destroy", None)
        if h and h.value and destroy is not None:
            destroy(h)
            self._h = None

    def value(self, x, stream=None):
        """V for fp32 features [n, 198] (generic fp32 FMA path)."""
        x = torch.as_tensor(x, dtype=torch.float32)
        if not x.is_cuda:
            x = x.cuda()
        x = x.contiguous().view(-1, 198)
        out = torch.empty((x.shape[0],), dtype=torch.float32, device=x.device)
        check(lib().bgx_value(self._h, ptr(x), x.shape[0], ptr(out), stream_handle(stream)), "bgx_value")
        return out

    def value_boards(self, boards, player, stream=None):
        """V of get_board_features(board, player) via the fused split-fp16 MFMA kernel."""
        boards, player = _u8(boards).view(-1, 52), _u8(player).view(-1)
        require_cuda(boards, player)
        out = torch.empty((boards.shape[0],), dtype=torch.float32, device=boards.device)
        check(lib().bgx_value_boards(self._h, ptr(boards), ptr(player), boards.shape[0], ptr(out),
                                     stream_handle(stream)), "bgx_value_boards")
        return out

    def two_ply(self, boards, opponent, sample=0, seed=0, stream=None):
        """compute_weighted_opponent_response (two_ply.py:93-150) for afterstates
        [n, 52]; returns float64 W [n]. sample=0: exact mode; sample=50: the
        reference's random.sample of 50 replies for 1-1 / 2-2 / 3-3
        (two_ply.py:119-121), reproducible per seed."""
        boards, opponent = _u8(boards).view(-1, 52), _u8(opponent).view(-1)
        require_cuda(boards, opponent)
        out = torch.empty((boards.shape[0],), dtype=torch.float64, device=boards.device)
        check(lib().bgx_two_ply_sampled(self._h, ptr(boards), ptr(opponent), boards.shape[0], int(sample),
                                        int(seed), ptr(out), stream_handle(stream)), "bgx_two_ply_sampled")
        return out


def load_pth(path):
    """A reference checkpoint (torch.save of BackgammonPolicyNetwork.state_dict(),
    parameter_manager.py:115-151: fc1.weight / fc1.bias / value_head.weight /
    value_head.bias) -> dict of host fp32 W1, b1, w2, b2. Loaded with
    weights_only=True (no code from the file runs)."""
    sd = torch.load(path, map_location="cpu", weights_only=True)
    return dict(zip(("W1", "b1", "w2", "b2"), weights_from(sd)))
