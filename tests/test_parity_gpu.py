"""GPU parity tests: librtamd (gfx950 kernels, through the C-ABI) vs the CPU
oracle on the same inputs -- bit-exact for bounds, Morton codes, sorted
keys/indices, topology, escape links, AABBs, hits, counters and images
(hits are allowed 1 ulp, we require 0 and report it).
Parity vs upstream SoslanGM/gpu_raytracer is unpinned (code-less reference);
the oracle is pinned by tests/test_oracle.py."""
import numpy as np
import pytest

from conftest import bits, load_golden

pytestmark = pytest.mark.gpu
SENT = 0xFFFFFFFF


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    return rt


def soup(oracle, n, seed=1):
    return oracle.soup(n, seed).reshape(-1, 9)


# ------------------------------------------------------------------ semantics probes
def test_single_hip_runtime(R):
    maps = open("/proc/self/maps").read()
    libs = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(libs) == 1, libs


def test_device_minmax_semantics(R, oracle):
    """The contract's fminf/fmaxf (v_min/v_max) == the oracle's restatement."""
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 1e-45, -1e-45, 3.4e38], np.float32)
    a, b = np.meshgrid(sp, sp, indexing="ij")
    rng = np.random.default_rng(0)
    a = np.concatenate([a.ravel(), rng.standard_normal(1000).astype(np.float32)])
    b = np.concatenate([b.ravel(), rng.standard_normal(1000).astype(np.float32)])
    mn, mx = R.stage_minmax(a, b)
    L = oracle.lib()
    emn = np.array([L.orc_fmin(float(x), float(y)) for x, y in zip(a, b)], np.float32)
    emx = np.array([L.orc_fmax(float(x), float(y)) for x, y in zip(a, b)], np.float32)
    nan = np.isnan(emn)
    assert np.array_equal(np.isnan(mn), nan)
    assert np.array_equal(bits(mn[~nan]), bits(emn[~nan]))
    nan = np.isnan(emx)
    assert np.array_equal(np.isnan(mx), nan)
    assert np.array_equal(bits(mx[~nan]), bits(emx[~nan]))


def test_device_intersect(R, oracle):
    tri = np.array([[-1, -1, 0, 1, -1, 0, -1, 1, 0]], np.float32)
    hit, tuv = R.stage_intersect([[0, 0, -1]], [[0, 0, 1]], tri, [np.inf])
    assert hit[0] and tuple(tuv[0]) == (1.0, 0.5, 0.5)
    rng = np.random.default_rng(3)
    n = 4096
    o = rng.standard_normal((n, 3)).astype(np.float32)
    d = rng.standard_normal((n, 3)).astype(np.float32)
    t = (rng.standard_normal((n, 9)) * 2).astype(np.float32)
    tb = np.where(rng.random(n) < 0.3, rng.random(n) * 3, np.inf).astype(np.float32)
    hit, tuv = R.stage_intersect(o, d, t, tb)
    for i in range(n):
        h, tt, uu, vv = oracle.intersect_tri(o[i], d[i], t[i], tb[i])
        assert hit[i] == h, i
        if h:
            assert np.array_equal(bits(tuv[i]), bits(np.array([tt, uu, vv], np.float32))), i
    assert hit.sum() > 100


# ------------------------------------------------------------------ stages
@pytest.mark.parametrize("n", [0, 1, 5, 255, 256, 257, 100000, 1000003])
def test_stage_bounds_morton(R, oracle, n):
    tris = soup(oracle, n, 4)
    lo, hi, inv = R.stage_bounds(tris)
    elo, ehi, einv = oracle.centroid_bounds(tris)
    assert np.array_equal(bits(lo), bits(elo)) and np.array_equal(bits(hi), bits(ehi))
    assert np.array_equal(bits(inv), bits(einv))
    if n:
        k, v = R.stage_morton(tris, lo, inv)
        ek, ev = oracle.morton(tris, elo, einv)
        assert np.array_equal(k, ek) and np.array_equal(v, ev)


def _keys(kind, n, rng):
    return {
        "random": rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
        "morton30": rng.integers(0, 2**30, n, dtype=np.uint64).astype(np.uint32),
        "equal": np.full(n, 0x12345678, np.uint32),
        "sorted": np.arange(n, dtype=np.uint32),
        "reversed": np.arange(n, dtype=np.uint32)[::-1].copy(),
        "onebucket": (rng.integers(0, 256, n) << 16).astype(np.uint32),
        "fewkeys": rng.integers(0, 3, n).astype(np.uint32) * 0x01010101,
    }[kind]


@pytest.mark.parametrize("n", [2, 3, 4095, 4096, 4097, 12289, 250000, 1 << 20])
@pytest.mark.parametrize("kind", ["random", "morton30", "equal", "sorted", "reversed", "onebucket", "fewkeys"])
def test_stage_sort(R, n, kind):
    rng = np.random.default_rng(n)
    keys = _keys(kind, n, rng)
    vals = rng.permutation(n).astype(np.uint32)
    k, v = R.stage_sort(keys, vals)
    o = np.argsort(keys, kind="stable")
    assert np.array_equal(k, keys[o])
    assert np.array_equal(v, vals[o])


@pytest.mark.parametrize("n", [2, 3, 8, 1000, 65537])
def test_stage_topology(R, oracle, n):
    tris = soup(oracle, n, 9)
    b = oracle.build(tris)
    keys = b["keys"]
    left, right, rlo, rhi, parent = oracle.karras(keys)
    esc = oracle.escape(n, left, right, parent)
    topo, par, lesc = R.stage_topology(keys)
    assert np.array_equal(topo[:, 0], left)
    assert np.array_equal(topo[:, 1], esc[: n - 1])
    assert np.array_equal(topo[:, 2], rlo) and np.array_equal(topo[:, 3], rhi)
    assert np.array_equal(par, parent)
    assert np.array_equal(lesc[: n - 1], esc[n - 1: 2 * n - 2])


def test_topology_fig4(R):
    g = load_golden("karras8.npz")
    topo, par, lesc = R.stage_topology(g["keys"])
    assert np.array_equal(topo[:, 0], g["left"]) and np.array_equal(topo[:, 1], g["esc"][:7])
    assert np.array_equal(par, g["parent"])
    assert np.array_equal(lesc[:7], g["esc"][7:14])


# ------------------------------------------------------------------ full build
def _compare_build(R, oracle, tris):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    with R.Scene.from_soup(tris) as s:
        s.build()
        got = s.read_bvh()
    exp = oracle.build(tris)
    for f in ("lo", "hi", "inv"):
        assert np.array_equal(bits(got[f]), bits(exp[f])), f
    assert np.array_equal(got["keys"], exp["keys"])
    assert np.array_equal(got["vals"], exp["vals"])
    assert np.array_equal(got["parent"], exp["parent"])
    g, e = got["nodes"], exp["nodes"]
    assert np.array_equal(g["a"], e["a"])
    assert np.array_equal(g["esc"], e["esc"])
    assert np.array_equal(bits(g["lo"]), bits(e["lo"]))
    assert np.array_equal(bits(g["hi"]), bits(e["hi"]))
    return got


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8, 100, 1023, 1024, 1025, 2047, 2048, 2049, 3073, 4096 * 3 + 7, 50000])
def test_build_parity_small(R, oracle, n):
    _compare_build(R, oracle, soup(oracle, n, n))


@pytest.mark.parametrize("n", [300000, 1000000])
def test_build_parity_large(R, oracle, n):
    _compare_build(R, oracle, soup(oracle, n, 1))


def test_build_parity_10m_sparse_table_path(R, oracle):
    """10M prims: 9766 refit blocks -> the global sparse-table crossing path."""
    _compare_build(R, oracle, soup(oracle, 10_000_000, 1))


def test_build_degenerate_inputs(R, oracle):
    rng = np.random.default_rng(7)
    one = soup(oracle, 1, 3)
    _compare_build(R, oracle, np.tile(one, (5000, 1)))                     # all identical -> equal keys
    flat = soup(oracle, 3000, 4).copy()
    flat[:, 2::3] = 0.25                                                    # zero extent in z -> inv_z = 0
    _compare_build(R, oracle, flat)
    clustered = (rng.random((20000, 9)) * 1e-3).astype(np.float32)
    clustered[:10] += 1000.0                                                # extreme outliers
    _compare_build(R, oracle, clustered)
    neg = -soup(oracle, 5000, 5)                                            # negative coordinates, -0
    _compare_build(R, oracle, neg)


SORT_DEFAULT = 2  # build.sort: the tile-bucketed gather sort


def _compare_sorts(R, tris):
    """The build with the tile-bucketed gather sort (build.sort = 2, the
    default for 2 <= n <= 12M), the MSB scatter + bucket sort (1) and the
    4-pass LSB sort (0) must give the same BVH; each scene's first build (the
    probe) and a second build alike."""
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    outs = []
    try:
        for mode, fuse in ((0, 1), (1, 1), (2, 1), (2, 0)):  # (2, 1): K0 + K1 fused where the grid fits
            R.config_set("build.sort", mode)
            R.config_set("build.fuse_k01", fuse)
            with R.Scene.from_soup(tris) as s:
                for _ in range(2):
                    s.build()
                    outs.append(s.read_bvh())
    finally:
        R.config_set("build.sort", SORT_DEFAULT)
        R.config_set("build.fuse_k01", 1)
    a = outs[0]
    for b in outs[1:]:
        assert np.array_equal(a["keys"], b["keys"])
        assert np.array_equal(a["vals"], b["vals"])
        assert np.array_equal(a["nodes"].view(np.uint32), b["nodes"].view(np.uint32))


@pytest.mark.parametrize("n", [2, 3, 4097, 70000, 1000000, 1400000, 2097152, 2097153, 3000017, 6000000, 10000000,
                               12000000])
def test_build_sort_paths_agree(R, oracle, n):
    _compare_sorts(R, soup(oracle, n, 11))


def test_build_sort_paths_agree_clustered(R, oracle):
    """Buckets beyond one LDS sort (2048 keys): the chunked path."""
    rng = np.random.default_rng(12)
    c = (rng.random((30000, 9)) * 1e-3).astype(np.float32)
    c[:5] += 1.0                                   # outliers: the cluster is one top-10-bit bucket
    _compare_sorts(R, c)
    _compare_sorts(R, np.tile(soup(oracle, 1, 3), (9000, 1)))   # all keys equal
    mixed = soup(oracle, 60000, 13).copy()
    mixed[:25000] = mixed[:25000] * 1e-4 + 0.5     # one dense cell inside a uniform soup
    _compare_sorts(R, mixed)
    # n > 2^21 (1024-thread bucket sorts): a dense cell beyond one LDS sort
    # (12288 keys) takes the chunked path, the rest the LDS path
    big = soup(oracle, 2500000, 14).copy()
    big[:40000] = big[:40000] * 1e-4 + 0.25
    _compare_sorts(R, big)


def test_fused_k01_not_coresident_falls_back(R):
    """The fused K0 + K1's grid barrier must never hang and never fail a
    build: build.fuse_k01 = 2 forces the fused launch on
    a grid that cannot be co-resident (3M: 733 sort tiles against ~256
    resident blocks); the first round's blocks give up after their bounded
    wait (~100 ms), and the host discards that build and redoes it in the
    same call with the two-launch K0 + K1 -- bit-exact, fused_k01 == 0,
    fused_fallback == 1.  The barrier counter is left consistent: the same
    scene's next builds equal a fresh scene's, and so does a fused 1M build
    afterwards (whose barrier flag must not read as a stale timeout)."""
    rng = np.random.default_rng(31)
    big = rng.random((3_000_000, 9), dtype=np.float32)
    with R.Scene.from_soup(big) as ref:
        ref.build()
        exp = ref.read_bvh()
        # (unit-cube vertices: the centroids pile up in the middle, so this
        # scene's probe verdict is the LSB sort -- the redo must reach it too)
        exp_kind = ref.build_times().sort_kind
    # a uniform soup keeps the gather sort, so every build of it is fused
    with R.Scene.generate_soup(1_000_000, 5) as ref:
        ref.build()
        exp_small = ref.read_bvh()
        assert ref.build_times().fused_k01 == 1
    R.config_set("build.fuse_k01", 2)
    try:
        with R.Scene.from_soup(big) as s:
            s.build()  # falls back, no exception
            t = s.build_times()
            assert (t.fused_k01, t.fused_fallback, t.sort_kind) == (0, 1, exp_kind), t
            assert t.total > 50.0, t  # the discarded build's ~100-ms wait is part of what the call spent
            got = s.read_bvh()
            assert np.array_equal(got["keys"], exp["keys"])
            assert np.array_equal(got["vals"], exp["vals"])
            assert np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32))
            R.config_set("build.fuse_k01", 1)
            for _ in range(2):
                s.build()
                t = s.build_times()
                assert (t.fused_k01, t.fused_fallback) == (0, 0), t
                got = s.read_bvh()
                assert np.array_equal(got["vals"], exp["vals"])
                assert np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32))
        with R.Scene.generate_soup(1_000_000, 5) as s:
            for _ in range(2):
                s.build()
                t = s.build_times()
                assert (t.fused_k01, t.fused_fallback) == (1, 0), t
                got = s.read_bvh()
                assert np.array_equal(got["nodes"].view(np.uint32), exp_small["nodes"].view(np.uint32))
    finally:
        R.config_set("build.fuse_k01", 1)


@pytest.mark.parametrize("n", [1000, 1_000_000])
def test_lsb_redo_branch(R, oracle, n):
    """the host's discard-and-redo branch for a gather
    bucket that overflows outside a probe build cannot be reached with real
    scenes (a scene's triangles never change), so debug.force_lsb_redo takes
    it: the redo runs the LSB sort, the scene keeps it, the BVH equals the
    oracle's, the stage times are the redo's and the total covers both."""
    tris = soup(oracle, n, 77)
    exp = oracle.build(tris)
    with R.Scene.from_soup(tris) as s:
        s.build()
        R.config_set("debug.force_lsb_redo", 1)
        R.config_set("build.stage_events", 1)
        try:
            s.build()
        finally:
            R.config_set("debug.force_lsb_redo", 0)
            R.config_set("build.stage_events", 0)
        t = s.build_times()
        assert (t.lsb_redo, t.sort_kind) == (1, 0), t
        stages = t.bounds + t.morton + t.sort + t.topology + t.refit + t.wide
        assert 0 < stages <= t.total, t
        _same_bvh(s.read_bvh(), exp)
        s.build()  # the scene keeps the LSB sort, no redo
        t = s.build_times()
        assert (t.lsb_redo, t.sort_kind) == (0, 0), t
        _same_bvh(s.read_bvh(), exp)


def _same_bvh(got, exp):
    assert np.array_equal(got["keys"], exp["keys"])
    assert np.array_equal(got["vals"], exp["vals"])
    g, e = got["nodes"], exp["nodes"]
    for f in ("a", "esc"):
        assert np.array_equal(g[f], e[f]), f
    for f in ("lo", "hi"):
        assert np.array_equal(bits(g[f]), bits(e[f])), f


@pytest.mark.parametrize("n", [1_000_000, 1_900_000, 2_000_000, 2_097_152, 2_097_153, 3_000_017, 10_000_000])
def test_uniform_soup_keeps_gather_sort(R, n):
    """a uniform soup's sort must not depend on n -- no LSB
    cliff where the mean bucket (n/1024) nears a fixed cap.  The gather
    sort's bucket capacity grows with n (mean + 16 sigma + 64, gather_shape),
    so every size up to 12M keeps it after its probe build; the 1M soup's
    K0 + K1 run as one launch."""
    with R.Scene.generate_soup(n, 7) as s:
        for _ in range(2):
            s.build()
            t = s.build_times()
            assert t.sort_kind == 2, (n, t)
        if n == 1_000_000:
            assert t.fused_k01 == 1, t


@pytest.mark.parametrize("sort", [1, 2])
@pytest.mark.parametrize("n", [1_000_000, 3_000_000])  # LDS bucket sort / the _big kernels (n > kMsbMaxN)
def test_clustered_scene_switches_sort(R, oracle, n, sort):
    """A scene whose first build finds an MSB bucket beyond one LDS sort -- a
    quarter of the soup in one tiny cell -- is sorted by the gated 4-pass LSB
    leg of that same build (launch_sort_probe) and by the LSB sort from then
    on (BuildBufs::sort_mode): every build equals the oracle, and none pays
    for one block sorting the dense cell (1.87 ms at 1M before the probe)."""
    rng = np.random.default_rng(5)
    t = rng.random((n, 9), dtype=np.float32)
    t[: n // 4] = 0.5 + rng.random((n // 4, 9), dtype=np.float32) * np.float32(1e-4)
    exp = oracle.build(t)
    R.config_set("build.sort", sort)
    try:
        with R.Scene.from_soup(rng.random((n, 9), dtype=np.float32)) as w:  # every build kernel loaded
            w.build()
        ms = []
        with R.Scene.from_soup(t) as s:
            for _ in range(3):
                ms.append(s.build())
                assert s.build_times().sort_kind == 0  # the verdict: LSB from the first build on
                got = s.read_bvh()
                assert np.array_equal(got["keys"], exp["keys"])
                assert np.array_equal(got["vals"], exp["vals"])
                assert np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32))
    finally:
        R.config_set("build.sort", SORT_DEFAULT)
    assert max(ms) < 1.0 * n / 1e6, ms


def _clustered_tris(oracle, scene):
    from gpu_raytracer_amd import scenes as S
    rng = np.random.default_rng(7)
    if scene == "hot":  # a soup plus 1500 small triangles in a cube of side 0.01: a 398-key bin
        c = rng.random((1500, 1, 3)).astype(np.float32) * 0.01 + 0.3
        h = (c + rng.standard_normal((1500, 3, 3)).astype(np.float32) * 1e-4).reshape(-1, 9)
        return np.ascontiguousarray(np.concatenate([soup(oracle, 60000, 3), h]), np.float32)
    if scene == "dup":  # 300 copies of each of 200 triangles: runs of 300 identical keys
        d = np.repeat(soup(oracle, 200, 5), 300, axis=0)
        return np.ascontiguousarray(np.concatenate([soup(oracle, 30000, 4), d]), np.float32)
    return np.ascontiguousarray(S.tris_for(scene), np.float32).reshape(-1, 9)


@pytest.mark.parametrize("scene,kind", [("bunny", 2), ("sponza", 2), ("hot", 2), ("dup", 1)])
def test_clustered_scenes_sort(R, oracle, scene, kind):
    """Clustered bins stay on the gather sort (r06): the bunny substitute
    (70K triangles; the poles of its lat-long sphere put up to 75 keys in one
    fine bin), the Sponza substitute (262K; a 2048-key bucket against a mean
    of 256, 32-key bins) and a soup with a 398-key bin take the gather's
    radix path for their hot buckets (gather_radix_sort), bit-exact.  Runs
    of 300 identical keys (duplicated triangles) flag the scene, which moves
    on to the MSB bucket sort (BuildBufs::gather_off).  Every build equals
    the oracle."""
    t = _clustered_tris(oracle, scene)
    exp = oracle.build(t)
    kinds = []
    with R.Scene.from_soup(t) as s:
        for _ in range(3):
            s.build()
            kinds.append(s.build_times().sort_kind)
            got = s.read_bvh()
            assert np.array_equal(got["keys"], exp["keys"])
            assert np.array_equal(got["vals"], exp["vals"])
            assert np.array_equal(got["nodes"].view(np.uint32), exp["nodes"].view(np.uint32))
    assert kinds == [kind] * 3, kinds


def test_build_repeat_and_rebuild(R, oracle):
    """Control words are re-armed between builds (zeroed per build)."""
    tris = soup(oracle, 70000, 2)
    exp = oracle.build(tris)
    with R.Scene.from_soup(tris) as s:
        for _ in range(3):
            s.build()
            got = s.read_bvh()
            assert np.array_equal(got["vals"], exp["vals"])
            assert np.array_equal(bits(got["nodes"]["lo"]), bits(exp["nodes"]["lo"]))


# ------------------------------------------------------------------ render
def _cam(R, view, w, h):
    return R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)


def _compare_render(R, oracle, tris, view, w, h, spp):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    exp = oracle.build(tris)
    cam = _cam(R, view, w, h)
    ocam = oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
    ehits, ecnt = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
    ergba = oracle.shade(ehits, w, h, spp)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render(cam, w, h, spp)
        cnt = s.render_counters(cam, w, h, spp)
    assert np.array_equal(hits["prim"], ehits["prim"])
    for f in ("t", "u", "v"):
        assert np.array_equal(bits(hits[f]), bits(ehits[f])), f
    assert np.array_equal(rgba, ergba)
    assert cnt[0] == ecnt[0] and cnt[1] == ecnt[1]
    return hits, cnt


def test_render_golden_soup1024(R):
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    g = load_golden("soup1024.npz")
    with R.Scene.from_soup(g["tris"]) as s:
        s.build()
        for (w, h, spp) in [(64, 48, 1), (32, 24, 3)]:
            tag = f"r{w}x{h}x{spp}_"
            cam = _cam(R, SOUP_VIEW, w, h)
            assert np.array_equal(bits(R.camera_array(cam)), bits(g[tag + "cam"]))
            hits, rgba, _ = s.render(cam, w, h, spp)
            assert np.array_equal(hits["prim"], g[tag + "prim"])
            for f in ("t", "u", "v"):
                assert np.array_equal(bits(hits[f]), bits(g[tag + f]))
            assert np.array_equal(rgba, g[tag + "rgba"])
            cnt = s.render_counters(cam, w, h, spp)
            assert np.array_equal(cnt, g[tag + "counters"])


def test_render_golden_cornell(R):
    from gpu_raytracer_amd.scenes import CORNELL_VIEW
    g = load_golden("cornell.npz")
    with R.Scene.from_soup(g["tris"]) as s:
        s.build()
        _, rgba, _ = s.render(_cam(R, CORNELL_VIEW, 256, 256), 256, 256, 1, hits=False)
        assert np.array_equal(rgba, g["r256x256x1_rgba"])
        hits, _, _ = s.render(_cam(R, CORNELL_VIEW, 64, 64), 64, 64, 1)
        assert np.array_equal(hits["prim"], g["r64x64x1_prim"])
        assert np.array_equal(bits(hits["t"]), bits(g["r64x64x1_t"]))


def test_render_golden_edge(R):
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    g = load_golden("edge.npz")
    for p, (w, h, spp) in [("n1_", (16, 16, 2)), ("n2_", (16, 16, 1)), ("dup64_", (16, 16, 1))]:
        with R.Scene.from_soup(g[p + "tris"]) as s:
            s.build()
            hits, rgba, _ = s.render(_cam(R, SOUP_VIEW, w, h), w, h, spp)
        tag = f"{p}r{w}x{h}x{spp}_"
        assert np.array_equal(hits["prim"], g[tag + "prim"]) and np.array_equal(rgba, g[tag + "rgba"])
        assert np.array_equal(bits(hits["t"]), bits(g[tag + "t"]))


@pytest.mark.parametrize("n,w,h,spp", [(0, 16, 16, 1), (1, 33, 17, 1), (20000, 160, 90, 2), (100000, 257, 129, 1)])
def test_render_parity(R, oracle, n, w, h, spp):
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    tris = soup(oracle, n, 5) if n else np.zeros((0, 9), np.float32)
    hits, _ = _compare_render(R, oracle, tris, SOUP_VIEW, w, h, spp)
    if n == 0:
        assert np.all(hits["prim"] == SENT) and np.all(np.isinf(hits["t"]))


def test_render_parity_presets(R, oracle):
    from gpu_raytracer_amd import scenes as S
    _compare_render(R, oracle, S.bunny_substitute_tris(), S.BUNNY_VIEW, 320, 180, 1)
    _compare_render(R, oracle, S.sponza_substitute_tris(), S.SPONZA_VIEW, 192, 108, 2)


def test_render_parity_headline_1m(R, oracle):
    """configs[2] at full size: 1M soup, 1920x1080x1 -- every hit bit-exact."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    tris = soup(oracle, 1_000_000, 1)
    hits, cnt = _compare_render(R, oracle, tris, SOUP_VIEW, 1920, 1080, 1)
    assert (hits["prim"] != SENT).sum() > 500000
    assert cnt[0] > 50_000_000


def test_tiled_render_matches_full(R, oracle):
    """Image-tile sharding (tile t -> rank t mod P) + unpack == one full render."""
    import torch
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    tris = soup(oracle, 50000, 8)
    w, h, spp = 200, 120, 2
    cam = _cam(R, SOUP_VIEW, w, h)
    with R.Scene.from_soup(tris) as s:
        s.build()
        _, full, _ = s.render(cam, w, h, spp, hits=False)
        for P in (1, 2, 3, 8):
            tmax = max(R.tiles_for_rank(w, h, r, P) for r in range(P))
            slabs = torch.zeros((P, max(tmax, 1) * 256), dtype=torch.int32, device="cuda")
            torch.cuda.synchronize()  # the zero fill (torch's stream) before the scene's stream writes
            for r in range(P):
                s.render_tiles_device(cam, w, h, spp, r, P, slabs[r].data_ptr())
            s.sync()
            img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
            R.unpack_tiles_device(slabs.data_ptr(), tmax, w, h, P, img.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(img.cpu().numpy().view(np.uint8), full), P


@pytest.mark.parametrize("px_sort", [1, 0, 2])
def test_tile_order_successive_frames(R, oracle, px_sort):
    """Longest-first tile dispatch from the previous frame's cost map (the
    default): the 1st frame runs row-major, later frames reordered -- every
    frame bit-identical to the oracle, full image and per-rank tiles alike,
    and a frame of another shape starts a fresh map.  px_sort: each tile's
    pixels dealt to lanes costliest first from the previous frame's per-pixel
    steps (1 = full frames, the default; 2 = also per-rank tiles; 0 = off);
    the 250x138 frames leave invalid pixels in the edge tiles' permutations."""
    tris = soup(oracle, 60000, 12)
    exp = oracle.build(tris)
    R.config_set("trace.tile_order", 1)
    R.config_set("trace.px_sort", px_sort)
    try:
        _successive_frames(R, oracle, s_tris=tris, exp=exp)
    finally:
        R.config_set("trace.px_sort", 1)


@pytest.mark.parametrize("n", [1, 5000])
def test_binary_variant_pixel_order_frames(R, oracle, n):
    """The binary k_trace instance (trace.variant = 2, and every scene with
    n < 2) has no traversal stack, yet its 256-thread full-frame blocks run the
    per-pixel order from the 2nd frame of an unchanged camera: its ranking
    LDS must be sized for it.  Three frames of one camera,
    each == the oracle."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    if n == 1:  # one large triangle across the view: hits and misses in every tile row
        tris = np.array([[0.1, 0.05, 0.5, 0.95, 0.3, 0.45, 0.35, 0.9, 0.55]], np.float32)
    else:
        tris = soup(oracle, n, 21)
    exp = oracle.build(tris)
    w, h, spp = 160, 96, 1
    ocam = oracle.camera_look_at(SOUP_VIEW.eye, SOUP_VIEW.at, SOUP_VIEW.up, SOUP_VIEW.vfov, w, h)
    eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
    er = oracle.shade(eh, w, h, spp)
    R.config_set("trace.variant", 2)
    R.config_set("trace.tile_order", 1)
    R.config_set("trace.px_sort", 1)
    try:
        with R.Scene.from_soup(tris) as s:
            s.build()
            cam = _cam(R, SOUP_VIEW, w, h)
            for _ in range(3):
                hits, rgba, _ = s.render(cam, w, h, spp)
                assert np.array_equal(rgba, er)
                assert np.array_equal(hits["prim"], eh["prim"])
                assert np.array_equal(bits(hits["t"]), bits(eh["t"]))
    finally:
        R.config_set("trace.variant", 0)


def _successive_frames(R, oracle, s_tris, exp):
    import torch
    from gpu_raytracer_amd.scenes import SOUP_VIEW
    tris = s_tris
    with R.Scene.from_soup(tris) as s:
        s.build()
        for (w, h, spp) in [(256, 144, 1), (256, 144, 1), (200, 120, 2), (256, 144, 1), (256, 144, 1),
                            (250, 138, 1), (250, 138, 1), (250, 138, 1)]:
            cam = _cam(R, SOUP_VIEW, w, h)
            ocam = oracle.camera_look_at(SOUP_VIEW.eye, SOUP_VIEW.at, SOUP_VIEW.up, SOUP_VIEW.vfov, w, h)
            eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
            er = oracle.shade(eh, w, h, spp)
            hits, rgba, _ = s.render(cam, w, h, spp)
            assert np.array_equal(rgba, er)
            assert np.array_equal(hits["prim"], eh["prim"])
            assert np.array_equal(bits(hits["t"]), bits(eh["t"]))
        w, h, spp, P = 250, 138, 1, 3
        cam = _cam(R, SOUP_VIEW, w, h)
        _, full, _ = s.render(cam, w, h, spp, hits=False)
        tmax = max(R.tiles_for_rank(w, h, r, P) for r in range(P))
        # per-rank maps: 3 successive frames of the SAME rank, so frames 2 and
        # 3 run reordered from that rank's own cost map (a scene keeps one
        # map per frame shape, and rank is part of the shape)
        for wg in (64, 256):
            R.config_set("trace.wg_tiles", wg)
            try:
                slabs = torch.zeros((P, tmax * 256), dtype=torch.int32, device="cuda")
                torch.cuda.synchronize()  # the zero fill (torch's stream) before the scene's stream writes
                for r in range(P):
                    first = None
                    for frame in range(3):
                        s.render_tiles_device(cam, w, h, spp, r, P, slabs[r].data_ptr())
                        s.sync()
                        cur = slabs[r].cpu().numpy().copy()
                        if first is None:
                            first = cur
                        assert np.array_equal(cur, first), (wg, r, frame)
                img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
                R.unpack_tiles_device(slabs.data_ptr(), tmax, w, h, P, img.data_ptr())
                torch.cuda.synchronize()
                assert np.array_equal(img.cpu().numpy().view(np.uint8), full), wg
            finally:
                R.config_set("trace.wg_tiles", 64)


def test_tile_order_moving_camera(R, oracle):
    """A camera that moves every frame (the bench's orbit): the tile order
    comes from the previous frame's map, the pixel order is skipped while
    the camera moves and resumes when it stops -- every frame == the oracle."""
    import math
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = soup(oracle, 40000, 14)
    exp = oracle.build(tris)
    w, h = 240, 136
    with R.Scene.from_soup(tris) as s:
        s.build()
        for i in (0, 1, 2, 3, 3, 3):
            a = math.radians(2.0 * i)
            ex, ez = V.eye[0] - V.at[0], V.eye[2] - V.at[2]
            eye = (V.at[0] + ex * math.cos(a) - ez * math.sin(a), V.eye[1],
                   V.at[2] + ex * math.sin(a) + ez * math.cos(a))
            cam = R.camera_look_at(eye, V.at, V.up, V.vfov, w, h)
            ocam = oracle.camera_look_at(eye, V.at, V.up, V.vfov, w, h)
            eh, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, 1)
            hits, rgba, _ = s.render(cam, w, h, 1)
            assert np.array_equal(rgba, oracle.shade(eh, w, h, 1)), i
            assert np.array_equal(bits(hits["t"]), bits(eh["t"])), i


@pytest.mark.parametrize("n", [140_000, 300_000])
def test_crossing_ranges_at_group_boundaries(R, oracle, n):
    """The crossing stage on crafted sorted keys whose subtrees cover exactly
    one whole group (64 refit blocks) of middle blocks, or sit inside one:
    at 140K (547 refit blocks) the small-scene LDS tree over every block
    total, at 300K (1172 blocks) the group tables (k_group_tables).
    rt_stage_refit's every node record == boxes unioned in numpy over each
    node's leaf range (a sparse table), with the oracle's topology and escape
    links.  (A middle range of exactly 64 blocks once took a non-existent
    in-group level.)"""
    cuts = [32_356, 65_587, 98_057, 114_692, 131_072 + 77, 196_608 - 5, 262_144 + 3]
    segs = [0] + [c for c in cuts if c < n] + [n]  # segment j: keys j << 24 | offset
    keys = np.zeros(n, np.uint32)
    for j in range(len(segs) - 1):
        keys[segs[j]:segs[j + 1]] = (j << 24) | np.arange(segs[j + 1] - segs[j], dtype=np.uint32)
    vals = np.arange(n, dtype=np.uint32)
    tris = soup(oracle, n, 5)
    nodes = R.stage_refit(keys, vals, tris)
    left, right, rlo, rhi, parent = oracle.karras(keys)
    esc = oracle.escape(n, left, right, parent)
    t = tris.reshape(n, 3, 3)
    blo, bhi = t.min(axis=1), t.max(axis=1)
    # sparse tables of the leaf boxes, then every internal node's range union
    tabs_lo, tabs_hi = [blo], [bhi]
    k = 1
    while (1 << k) <= n:
        h = 1 << (k - 1)
        a, b = tabs_lo[-1], tabs_hi[-1]
        tabs_lo.append(np.minimum(a[:-h], a[h:]))
        tabs_hi.append(np.maximum(b[:-h], b[h:]))
        k += 1
    ln = (rhi - rlo + 1).astype(np.int64)
    lv = np.floor(np.log2(ln)).astype(np.int64)
    exp_lo = np.zeros((n - 1, 3), np.float32)
    exp_hi = np.zeros((n - 1, 3), np.float32)
    for s in np.unique(lv):
        sel = np.nonzero(lv == s)[0]
        a0, a1 = rlo[sel].astype(np.int64), (rhi[sel].astype(np.int64) - (1 << s) + 1)
        exp_lo[sel] = np.minimum(tabs_lo[s][a0], tabs_lo[s][a1])
        exp_hi[sel] = np.maximum(tabs_hi[s][a0], tabs_hi[s][a1])
    g = nodes[: n - 1]
    assert np.array_equal(g["a"], left)
    assert np.array_equal(g["esc"], esc[: n - 1])
    assert np.array_equal(bits(g["lo"]), bits(exp_lo))
    assert np.array_equal(bits(g["hi"]), bits(exp_hi))
    lf = nodes[n - 1:]
    assert np.array_equal(lf["a"], vals) and np.array_equal(lf["esc"], esc[n - 1:])
    assert np.array_equal(bits(lf["lo"]), bits(blo)) and np.array_equal(bits(lf["hi"]), bits(bhi))
