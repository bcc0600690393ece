"""Shared pytest setup: the `gpu` marker, import paths and golden fixtures."""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mlp-ppo-2ply-multi_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libbgx.so on cuda:0)")


_CACHE = {}


def golden(name):
    """All arrays of a golden .npz, loaded once (NpzFile re-reads per access)."""
    if name not in _CACHE:
        with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
            _CACHE[name] = {k: z[k] for k in z.files}
    return _CACHE[name]


@pytest.fixture(scope="session")
def weights_seed0():
    d = golden("weights_seed0.npz")
    return {k: d[k] for k in ("W1", "b1", "w2", "b2")}


@pytest.fixture(scope="session")
def weights_ckpt():
    d = golden("weights_ckpt2100000.npz")
    return {k: d[k] for k in ("W1", "b1", "w2", "b2")}
