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


# Task accounting (DESIGN.md "The r02 8-ary wrong-hit record"): the oracle's
# traces start up to 15 worker threads per call, and a GPU box caps a job's
# tasks (threads count).  The session reports the most threads this process
# held after any test and the cgroup's task limit, so a run shows how close
# the suite came to the cap.
_max_threads = [0, ""]


def _threads():
    try:
        with open("/proc/self/status") as f:
            for line in f:
                if line.startswith("Threads:"):
                    return int(line.split()[1])
    except OSError:
        pass
    return 0


def pytest_runtest_teardown(item):
    t = _threads()
    if t > _max_threads[0]:
        _max_threads[0], _max_threads[1] = t, item.nodeid


def pytest_terminal_summary(terminalreporter):
    lim = "unknown"
    for p in ("/sys/fs/cgroup/pids.max", "/sys/fs/cgroup/pids/pids.max"):
        try:
            with open(p) as f:
                lim = f.read().strip()
            break
        except OSError:
            pass
    terminalreporter.write_line(f"[tasks] most threads in this process after a test: {_max_threads[0]} "
                                f"({_max_threads[1]}); cgroup pids.max: {lim}")
