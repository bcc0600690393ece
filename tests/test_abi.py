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
    assert L.bgx_abi_version() == 4
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
