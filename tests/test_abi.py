"""CPU checks of the boundary: libbgx.so loads, exports every entry point
declared in include/bgx.h, the ctypes table matches, and ops fail loudly
without a GPU (there is no CPU fallback)."""
import os
import re
import subprocess

import pytest

from conftest import REPO, PKG

HEADER = os.path.join(REPO, "include", "bgx.h")
LIB = os.path.join(PKG, "bgx", "libbgx.so")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(bgx_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    return LIB


def test_every_declared_symbol_is_exported(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\sT\s(bgx_\w+)", out))
    names = declared()
    assert len(names) >= 20
    missing = [n for n in names if n not in exported]
    assert not missing, missing


def test_ctypes_table_covers_header(built):
    from bgx._lib import SIGNATURES
    assert set(declared()) == set(SIGNATURES)


def test_loads_without_gpu_and_reports_version(built):
    import bgx
    L = bgx.lib()
    assert L.bgx_abi_version() == 10
    assert L.bgx_last_error() is not None


def test_ops_fail_loudly_without_gpu(built):
    import numpy as np
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from bgx import BgxError, ops
    with pytest.raises((BgxError, RuntimeError, AssertionError)):
        ops.movegen(np.zeros((1, 52), np.uint8), np.zeros(1, np.uint8), np.ones((1, 2), np.uint8))


def test_argument_errors_cross_abi_as_codes(built):
    import bgx
    L = bgx.lib()
    assert L.bgx_movegen(None, None, None, -1, None, None, 0, None) == -1
    assert b"n=-1" in L.bgx_last_error()
    assert L.bgx_encode(None, None, 5, None, 7, None) == -1
    assert L.bgx_encode_packed(None, 5, None, 3, None) == -1
    assert L.bgx_encode_packed(None, 5, None, 0, None) == -1   # null pointers, no device touched
    assert L.bgx_step(None, 1, None) == -1


def test_engine_config_limits_cross_abi_as_codes(built):
    """bgx_engine_create rejects configurations the kernels cannot hold, before
    touching a device: max_legal > 512 on the phased engine (the select
    kernel's per-lane score row), > 2048 on the fused one, max_steps > 511
    (the record's step field), ring outside max_steps+1 .. 65536."""
    import ctypes
    import bgx
    from bgx._lib import Config
    L = bgx.lib()
    out = ctypes.c_void_p()
    cases = [dict(max_legal=1024, fused=0), dict(max_legal=1024, ply=2), dict(max_legal=4096, fused=1),
             dict(max_steps=600, ring=2048), dict(ring=100), dict(ring=1 << 17)]
    for kw in cases:
        cfg = Config()
        L.bgx_config_default(ctypes.byref(cfg))
        for k, v in kw.items():
            setattr(cfg, k, v)
        assert L.bgx_engine_create(0, ctypes.byref(cfg), ctypes.byref(out)) == -1, kw
        if kw.get("max_legal") == 1024:
            assert b"max_legal=1024 > 512" in L.bgx_last_error()


def test_config_default_matches_header(built):
    import ctypes
    import bgx
    from bgx._lib import Config
    cfg = Config()
    bgx.lib().bgx_config_default(ctypes.byref(cfg))
    assert (cfg.lanes, cfg.ply, cfg.k_top, cfg.max_steps, cfg.max_legal, cfg.ring) == (4096, 1, 4, 300, 500, 1024)
    assert abs(cfg.alpha - 1.0) < 1e-7 and abs(cfg.beta - 0.9) < 1e-7 and cfg.fused == 1


def _host_check(boards, player=None, dice=None):
    import ctypes
    import numpy as np
    import bgx
    b = np.ascontiguousarray(np.asarray(boards, np.uint8).reshape(-1, 52))
    p = None if player is None else np.ascontiguousarray(np.asarray(player, np.uint8).reshape(-1))
    d = None if dice is None else np.ascontiguousarray(np.asarray(dice, np.uint8).reshape(-1, 2))
    f, first = ctypes.c_uint32(0), ctypes.c_int32(-1)
    rc = bgx.lib().bgx_check_boards_host(b.ctypes.data, None if p is None else p.ctypes.data,
                                         None if d is None else d.ctypes.data, len(b), ctypes.byref(f),
                                         ctypes.byref(first))
    assert rc == 0
    return f.value, first.value


def domain_cases():
    """(name, board, player, dice, expected BGX_BADF_* bits): one case per
    rejection rule of include/bgx.h plus legal inputs (the initial position,
    a bear-off, a game-over and a fewer-than-15 board are all accepted)."""
    import numpy as np
    from conftest import golden
    init = golden("movegen_cases.npz")["boards"][0].copy()
    cases = [("initial", init, 0, (3, 1), 0)]
    go = init.copy(); go[0:24] = 0; go[50] = 15
    cases.append(("game over", go, 0, (6, 6), 0))
    few = np.zeros(52, np.uint8); few[3] = 2; few[24 + 20] = 1
    cases.append(("fewer than 15", few, 1, (1, 2), 0))
    both = init.copy(); both[24 + 0] = 1; both[47] = 1   # P2 takes a checker onto P1's point 0 (P1 has 2 there)
    cases.append(("shared point", both, 0, (3, 1), 1))
    tot = init.copy(); tot[2] = 1                      # P1: 16 checkers
    cases.append(("16 checkers", tot, 0, (3, 1), 2))
    big = np.zeros(52, np.uint8); big[0] = 16          # a count above 15 (and 16 checkers)
    cases.append(("count 16", big, 0, (3, 1), 2 | 4))
    hi = init.copy(); hi[51] = 0x20                    # a byte above 15 in the off field
    cases.append(("byte 32", hi, 0, (3, 1), 2 | 4))
    cases.append(("die 0", init, 0, (0, 3), 8))
    cases.append(("die 7", init, 1, (4, 7), 8))
    cases.append(("player 2", init, 2, (3, 1), 16))
    return cases


@pytest.mark.parametrize("k", range(10))
def test_domain_rule_each_rejection_host(built, k):
    """bgx_check_boards_host applies the same rule (bgx_domain.h) as the
    device check every stateless entry point runs; each rule on its own."""
    name, b, p, d, want = domain_cases()[k]
    f, first = _host_check(b, [p], [d])
    assert f == want, name
    assert first == (0 if want else -1), name


def test_domain_rule_first_bad_index_and_unchecked_fields(built):
    import numpy as np
    cases = domain_cases()
    boards = np.stack([c[1] for c in cases])
    players = np.array([c[2] for c in cases], np.uint8)
    dice = np.array([c[3] for c in cases], np.uint8)
    f, first = _host_check(boards, players, dice)
    assert f == 1 | 2 | 4 | 8 | 16 and first == 3
    # player / dice not given: only the board rules apply
    f, first = _host_check(boards[[0, 7, 9]], None, None)
    assert f == 0 and first == -1


def test_domain_check_host_argument_errors(built):
    import bgx
    L = bgx.lib()
    assert L.bgx_check_boards_host(None, None, None, -1, None, None) == -1
    assert L.bgx_check_boards(None, None, None, 3, None, None, None) == -1
