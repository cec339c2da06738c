"""GPU test of the device BVH exchange (SURVEY.md §8(e) "rank 0 builds and
broadcasts"): a prepared-but-unbuilt scene whose BVH sections are filled from
a built one (standing in for the RCCL broadcast on one GPU) renders
bit-identically to the builder."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    return rt


def test_bvh_sections_copy_renders_identically(R, oracle):
    import torch
    from gpu_raytracer_amd import dist as D
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = oracle.soup(20000, 61).reshape(-1, 9)
    dev = torch.device("cuda", 0)
    with R.Scene.from_soup(tris) as a, R.Scene.from_soup(tris) as b:
        with pytest.raises(R.RtError):
            b.device_sections()                      # not prepared yet
        a.build()
        b.prepare()
        secs_a, secs_b = a.device_sections(), b.device_sections()
        n = len(tris)
        assert [nb for _, nb in secs_a] == [nb for _, nb in secs_b]
        assert [nb for _, nb in secs_a][1:] == [4 * n, 4 * n, 32 * (2 * n - 1), 48 * n, 64 * (n - 1)]
        with pytest.raises(R.RtError):
            cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, 64, 48)
            b.render(cam, 64, 48, 1)                 # prepared is not built
        for ta, tb in zip(D.bvh_tensors(a, dev), D.bvh_tensors(b, dev)):
            assert ta.data_ptr() != tb.data_ptr()
            tb.copy_(ta)
        b.mark_built()
        cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, 160, 96)
        ha, ia, _ = a.render(cam, 160, 96, 2)
        hb, ib, _ = b.render(cam, 160, 96, 2)
        assert np.array_equal(ia, ib)
        assert np.array_equal(ha.view(np.uint32), hb.view(np.uint32))
        ra, rb = a.read_bvh(), b.read_bvh()
        for k in ("keys", "vals", "parent"):
            assert np.array_equal(ra[k], rb[k])
        assert np.array_equal(a.read_wide(), b.read_wide())
