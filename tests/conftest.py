import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) GPU")


def _make(path, target):
    r = subprocess.run(["make", "-C", path, target], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stdout + r.stderr)


@pytest.fixture(scope="session")
def oracle_lib():
    if not os.path.exists(os.path.join(REPO, "oracle", "liboracle.so")):
        _make(os.path.join(REPO, "oracle"), "oracle")
    from oracle import core
    return core


@pytest.fixture(scope="session")
def engine_lib():
    """The product's C-ABI library, built in-tree if needed (no GPU required to load it)."""
    if not os.path.exists(os.path.join(PKG, "libuttt_engine.so")):
        _make(PKG, "all")
    from uttt_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def uttt_cpp_mod(engine_lib):
    import uttt_cpp
    return uttt_cpp


_GOLDEN_CACHE = {}


def golden(name):
    """Fixture arrays as a dict (NpzFile re-decompresses on every item access)."""
    import numpy as np
    if name not in _GOLDEN_CACHE:
        with np.load(os.path.join(GOLDEN, name)) as z:
            _GOLDEN_CACHE[name] = {k: z[k] for k in z.files}
    return _GOLDEN_CACHE[name]
