"""bench.py's multi-rank launch must end, whatever a rank does (VERDICT r02
"What's weak" 7): `bench.py --gpus N` supervises its rank processes with a
deadline and kills the rest once one fails; --pg-timeout bounds a stuck
collective; the BVH broadcast and distributed-build legs are opt-in
(--extras), so the headline line never waits on them.

CPU tests drive the supervisor with stand-in rank processes (one hangs, one
fails); the GPU tests run the real bench with 2 ranks over gloo on one GPU:
the gathered image must have the N=1 CRC, and a rank hung in the --extras
leg must make the run fail within its deadline instead of hanging."""
import os
import subprocess
import sys
import time

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

HEADLINE_CRC = 4209804860  # soup-1M 1920x1080x1, static camera (every N, bit-exact tiles)


def _kids(*codes_or_sleeps):
    out = []
    for c in codes_or_sleeps:
        prog = f"import time, sys; time.sleep({c[1]}); sys.exit({c[0]})"
        out.append(subprocess.Popen([sys.executable, "-c", prog]))
    return out


def test_supervise_all_ok():
    assert bench.supervise(_kids((0, 0.1), (0, 0.3)), deadline_s=30) == 0


def test_supervise_deadline_kills_hung_ranks():
    t0 = time.monotonic()
    procs = _kids((0, 600), (0, 600))
    rc = bench.supervise(procs, deadline_s=2.0)
    assert rc == 124
    assert time.monotonic() - t0 < 10
    assert all(p.poll() is not None for p in procs)


def test_supervise_failed_rank_ends_the_run():
    t0 = time.monotonic()
    procs = _kids((3, 0.1), (0, 600))
    rc = bench.supervise(procs, deadline_s=600, grace_s=1.0)
    assert rc == 3
    assert time.monotonic() - t0 < 10
    assert all(p.poll() is not None for p in procs)


def _bench(args, timeout):
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    return p, time.monotonic() - t0


@pytest.mark.gpu
def test_bench_two_ranks_gloo_crc():
    import json
    p, _ = _bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "3", "--warmup", "1", "--no-extra",
                   "--no-cpu-baseline", "--deadline", "240"], timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["image_crc32"] == HEADLINE_CRC
    assert line["bvh_exchange"] is None and line["distributed_build"] is None


@pytest.mark.gpu
def test_bench_hung_rank_fails_within_deadline():
    p, dt = _bench(["--gpus", "2", "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--no-extra",
                    "--no-cpu-baseline", "--extras", "--inject-hang", "1", "--pg-timeout", "30",
                    "--deadline", "120"], timeout=300)
    assert p.returncode != 0
    assert dt < 150, dt
