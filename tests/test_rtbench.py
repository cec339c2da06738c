"""rtbench, the C++ command-line driver: built by
build() against the C-ABI only.  CPU: usage, the loud RT_EDEVICE refusal
without a GPU, and its scene generators restating scenes.py bit for bit
(through --save-soup, which runs before the build).  GPU: a config-3 run
reports a sane JSON line, and a dumped Cornell frame equals the oracle's."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

EXE = os.path.join(ROOT, "gpu_raytracer_amd", "bin", "rtbench")


@pytest.fixture(scope="module")
def exe(rt):
    if not os.path.exists(EXE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "gpu_raytracer_amd"), "bin/rtbench"], check=True)
    return EXE


def _run(exe, *args, timeout=300):
    p = subprocess.run([exe, *args], capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout.strip().splitlines()


def test_usage(exe):
    rc, out = _run(exe, "--help")
    assert rc == 0 and out[0].startswith("usage: rtbench")
    rc, _ = _run(exe, "--mode", "nonsense")
    assert rc == 2


@pytest.mark.parametrize("scene", ["cornell", "bunny", "sponza"])
def test_scene_generators_match_python(exe, rt, tmp_path, scene):
    from gpu_raytracer_amd import scenes as S
    path = str(tmp_path / f"{scene}.rtsoup")
    _run(exe, "--scene", scene, "--save-soup", path)  # written before the build
    with rt.Scene.load_soup(path) as s:
        got = s.tris()
    exp = np.ascontiguousarray(S.tris_for(scene), np.float32).reshape(-1, 9)
    assert got.shape == exp.shape
    assert np.array_equal(got.view(np.uint32), exp.view(np.uint32))


def test_no_gpu_refusal(exe, rt):
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible")
    rc, out = _run(exe, "--config", "3", "--n", "1000")
    assert rc == 1
    j = json.loads(out[-1])
    assert j["status"] == "error" and j["code"] == -4  # RT_EDEVICE


@pytest.mark.gpu
def test_config3_json(exe, rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    rc, out = _run(exe, "--config", "3", "--frames", "5", "--warmup", "2", "--orbit", "0.25")
    assert rc == 0, out
    j = json.loads(out[-1])
    assert j["status"] == "ok" and j["n_tris"] == 1_000_000 and j["res"] == [1920, 1080]
    assert 0 < j["frame_ms_best"] <= j["frame_ms_median"] < 50 and j["build_ms"] > 0
    assert j["mrays_per_s"] > 100


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [1])
def test_cornell_dump_matches_oracle(exe, rt, oracle, tmp_path, gpus):
    from gpu_raytracer_amd import scenes as S
    w, h = 96, 80
    ppm = str(tmp_path / "c.ppm")
    rc, out = _run(exe, "--scene", "cornell", "--res", f"{w}x{h}", "--frames", "1", "--warmup", "0",
                   "--gpus", str(gpus), "--dump", ppm)
    assert rc == 0, out
    tris = np.ascontiguousarray(S.cornell_tris(), np.float32).reshape(-1, 9)
    V = S.CORNELL_VIEW
    b = oracle.build(tris)
    cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, _ = oracle.trace(b["nodes"], tris, cam, w, h, 1)
    er = oracle.shade(eh, w, h, 1).reshape(h, w, 4)[:, :, :3]
    data = open(ppm, "rb").read()
    header = b"P6\n%d %d\n255\n" % (w, h)
    assert data.startswith(header)
    img = np.frombuffer(data[len(header):], np.uint8).reshape(h, w, 3)
    assert np.array_equal(img, er)
