"""Shared pytest setup.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on the CPU container (``-m "not gpu"``).
The C oracle (oracle/, TEST INFRASTRUCTURE) is built on demand here.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    if not os.path.exists(O._LIB_PATH):
        O.build_oracle()
    O.lib()
    return O


@pytest.fixture(scope="session")
def rt():
    import gpu_raytracer_amd as R
    if not os.path.exists(R._lib.LIB_PATH):
        R.build_library()
    R.lib()
    return R


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def bits(a):
    """Bit pattern view for exact float comparison."""
    a = np.ascontiguousarray(a)
    if a.dtype == np.float32:
        return a.view(np.uint32)
    return a
