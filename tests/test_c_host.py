"""The C host of INTEGRATION.md (tests/c/rt_host.c): a plain C program linked
against librtamd.so, no Python in its process.  On the GPU its frame must be
byte-identical to the CPU oracle's (hits and RGBA); without a GPU it must
fail loudly with RT_EDEVICE (no CPU fallback)."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, bits

HOST = os.path.join(ROOT, "tests", "c", "build", "rt_host")


@pytest.fixture(scope="module")
def host(rt):
    if not os.path.exists(HOST):  # normally prebuilt by __graft_entry__.build()
        subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "c")], check=True, capture_output=True)
    return HOST


def _run(host, tmp_path, n, seed, w, h, spp, ngpus):
    a, b = tmp_path / "img.rgba", tmp_path / "img.hits"
    r = subprocess.run([host, str(n), str(seed), str(w), str(h), str(spp), str(ngpus), str(a), str(b)],
                       capture_output=True, text=True, timeout=120)
    return r, a, b


def test_c_host_without_gpu(rt, host, tmp_path):
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible; covered by test_c_host_matches_oracle")
    r, _, _ = _run(host, tmp_path, 100, 1, 8, 8, 1, 1)
    assert r.returncode == 3 and r.stdout.split()[0] == "-4", (r.stdout, r.stderr)
    assert "no CPU path" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("n,w,h,spp", [(4096, 96, 64, 1), (100000, 320, 180, 2)])
def test_c_host_matches_oracle(rt, oracle, host, tmp_path, n, w, h, spp):
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    r, a, b = _run(host, tmp_path, n, 1, w, h, spp, 1)
    assert r.returncode == 0, (r.stdout, r.stderr)
    tris = oracle.soup(n, 1).reshape(-1, 9)
    exp = oracle.build(tris)
    cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, cam, w, h, spp)
    got_hits = np.fromfile(b, dtype=eh.dtype)
    assert np.array_equal(bits(got_hits["t"]), bits(eh["t"]))
    assert np.array_equal(got_hits["prim"], eh["prim"])
    assert np.array_equal(bits(got_hits["u"]), bits(eh["u"])) and np.array_equal(bits(got_hits["v"]), bits(eh["v"]))
    assert np.array_equal(np.fromfile(a, np.uint8), oracle.shade(eh, w, h, spp))


@pytest.mark.gpu
def test_c_host_ngpus_beyond_devices(rt, host, tmp_path):
    r, _, _ = _run(host, tmp_path, 1000, 1, 32, 32, 1, rt.device_count() + 1)
    assert r.returncode == 3 and r.stdout.split()[0] == "-4", (r.stdout, r.stderr)
