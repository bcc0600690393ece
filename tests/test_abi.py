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
    assert L.bgx_abi_version() == 6
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
