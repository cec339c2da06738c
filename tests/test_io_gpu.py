"""GPU tests of the scene-I/O row: RTBVH1 cache
save/load, RTSOUP1 and OBJ ingest feeding the full build + trace, each
compared bit-for-bit with the direct path and the CPU oracle."""
import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    return rt


def _render(R, s, view, w, h, spp):
    cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    return s.render(cam, w, h, spp)


def test_bvh_cache_roundtrip(R, oracle, tmp_path):
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = oracle.soup(50000, 21).reshape(-1, 9)
    path = str(tmp_path / "soup.rtbvh")
    with R.Scene.from_soup(tris) as s:
        s.build()
        ref_bvh = s.read_bvh()
        ref_wide = s.read_wide()
        ref_hits, ref_rgba, _ = _render(R, s, V, 128, 96, 2)
        s.save_bvh(path)
    with R.Scene.from_soup(tris) as s:
        s.load_bvh(path)                       # no build
        got = s.read_bvh()
        for k in ("keys", "vals", "parent"):
            assert np.array_equal(got[k], ref_bvh[k]), k
        assert np.array_equal(got["nodes"].view(np.uint8), ref_bvh["nodes"].view(np.uint8))
        assert np.array_equal(s.read_wide(), ref_wide)
        hits, rgba, _ = _render(R, s, V, 128, 96, 2)
    assert np.array_equal(rgba, ref_rgba)
    assert np.array_equal(hits.view(np.uint32), ref_hits.view(np.uint32))


def test_bvh_cache_rejects(R, oracle, tmp_path):
    tris = oracle.soup(3000, 22).reshape(-1, 9)
    path = tmp_path / "a.rtbvh"
    with R.Scene.from_soup(tris) as s:
        with pytest.raises(R.RtError) as e:
            s.save_bvh(str(path))              # not built yet
        assert e.value.status == -1
        s.build()
        s.save_bvh(str(path))
    other = tris.copy()
    other[7, 3] += np.float32(1e-3)
    with R.Scene.from_soup(other) as s:
        with pytest.raises(R.RtError) as e:
            s.load_bvh(str(path))              # different triangles
        assert e.value.status == -1
    raw = path.read_bytes()
    for corrupt in (raw[:-10], raw + b"\0", raw[:8] + b"\x07" + raw[9:]):
        q = tmp_path / "bad.rtbvh"
        q.write_bytes(corrupt)
        with R.Scene.from_soup(tris) as s:
            with pytest.raises(R.RtError) as e:
                s.load_bvh(str(q))
            assert e.value.status == -3
    with R.Scene.from_soup(tris[:1]) as s:     # n = 1: no wide records
        s.build()
        s.save_bvh(str(tmp_path / "one.rtbvh"))
    with R.Scene.from_soup(tris[:1]) as s:
        s.load_bvh(str(tmp_path / "one.rtbvh"))


def test_rtsoup_and_obj_ingest_render_parity(R, oracle, tmp_path):
    """RTSOUP1 and OBJ (written with round-trip precision) give the same scene,
    the same BVH and the oracle's image."""
    from gpu_raytracer_amd import scenes as S
    tris = np.ascontiguousarray(S.bunny_substitute_tris(), np.float32).reshape(-1, 9)
    soup_path = str(tmp_path / "bunny.rtsoup")
    obj_path = tmp_path / "bunny.obj"
    with R.Scene.from_soup(tris) as s:
        s.save_soup(soup_path)
    lines = []
    for t in tris:
        for v in range(3):
            lines.append("v %.9g %.9g %.9g" % tuple(float(x) for x in t[3 * v:3 * v + 3]))
    lines += [f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}" for i in range(len(tris))]
    obj_path.write_text("\n".join(lines) + "\n")
    w, h = 160, 90
    V = S.BUNNY_VIEW
    ocam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    exp = oracle.build(tris)
    ehits, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, 1)
    ergba = oracle.shade(ehits, w, h, 1)
    for loader, arg in ((R.Scene.load_soup, soup_path), (R.Scene.load_obj, str(obj_path))):
        with loader(arg) as s:
            assert np.array_equal(bits(s.tris()), bits(tris))
            s.build()
            hits, rgba, _ = _render(R, s, V, w, h, 1)
        assert np.array_equal(rgba, ergba)
        assert np.array_equal(hits["prim"], ehits["prim"])
        assert np.array_equal(bits(hits["t"]), bits(ehits["t"]))
