"""GPU tests of the wide (4-ary) trace path: the K7w records and the three
trace variants, every one bit-exact against the CPU oracle's §9.7 binary
traversal (hits, images) -- including the hand-offs to the binary traversal
(forced stack overflows, rays with a zero direction component)."""
import numpy as np
import pytest

from conftest import bits

pytestmark = pytest.mark.gpu
SENT = 0xFFFFFFFF
LEAF = 0x80000000
VARIANTS = [0, 2]  # wide per pixel (default), binary per pixel (r06: the wide pool, 1, was removed)


@pytest.fixture(scope="module")
def R(rt):
    if rt.device_count() < 1:
        pytest.fail("no GPU visible to librtamd")
    yield rt
    rt.config_set("trace.variant", 0)
    rt.config_set("trace.stack_cap", 0)


def _decode_planes(rec):
    """Dequantized child planes of wide records (uint32[m, 16] 4-ary K7w or
    uint32[m, 24] 8-ary K7w8), computed as the kernel does: origin + q * 2^e
    rounded once (q * 2^e is exact, so the float32 add equals the kernel's
    fma).  Returns lo, hi as float32[m, 3, arity]."""
    W = 8 if rec.shape[1] == 24 else 4
    org = rec[:, 0:3].view(np.float32)
    meta = rec[:, 3]
    scale = ((meta[:, None] >> (8 * np.arange(3, dtype=np.uint32))) & 0xFF).astype(np.uint32) << 23
    scale = scale.view(np.float32)                              # [m, 3] = 2^e
    sh = (8 * np.arange(4, dtype=np.uint32))
    if W == 4:
        qlo = np.stack([rec[:, 4], rec[:, 5], rec[:, 6]], 1)[:, :, None]   # [m, 3, 1 word]
        qhi = np.stack([rec[:, 7], rec[:, 8], rec[:, 9]], 1)[:, :, None]
    else:  # two words per plane: qlo.x qlo.y qlo.z qhi.x qhi.y qhi.z at words 4..15
        qlo = rec[:, 4:10].reshape(-1, 3, 2)
        qhi = rec[:, 10:16].reshape(-1, 3, 2)
    ql = ((qlo[:, :, :, None] >> sh) & 0xFF).reshape(len(rec), 3, W).astype(np.float32)  # [m, 3, W]
    qh = ((qhi[:, :, :, None] >> sh) & 0xFF).reshape(len(rec), 3, W).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        lo = org[:, :, None] + ql * scale[:, :, None]
        hi = org[:, :, None] + qh * scale[:, :, None]
    return lo.astype(np.float32), hi.astype(np.float32)


def _layout(rec):
    """(arity, wild[m], valid mask[m], refs[m, arity]) of wide records."""
    meta = rec[:, 3]
    if rec.shape[1] == 24:
        wild = (meta & 0xFFFFFF) == 0xFFFFFF
        return 8, wild, meta >> 24, rec[:, 16:24]
    wild = ((meta >> 24) & 1).astype(bool)
    assert np.all(((meta & 0xFFFFFF) == 0xFFFFFF) == wild)  # wild records carry exponent bytes 255
    return 4, wild, (meta >> 28) & 0xF, rec[:, 10:14]


def _half_area(lo, hi):
    """csrc/build_kernels.hip half_area, same float32 operation order."""
    d = (hi - lo).astype(np.float32)
    return np.float32(np.float32(d[0] * d[1]) + np.float32(d[1] * d[2])) + np.float32(d[2] * d[0])


def _entries(X, a, esc, lo_e, hi_e, L0, arity=4):
    """Restatement of wide_entries (the greedy largest-surface cut): the
    record's entries in preorder."""
    def kids(c):
        L = a[c]
        return [L, esc[L]]  # escape of a left child = its right sibling
    ent = kids(X)
    for _ in range(arity - 2):
        best, ba = -1, None
        for i, c in enumerate(ent):
            if c < L0:
                ar = _half_area(lo_e[c], hi_e[c])
                if best < 0 or ar > ba:
                    best, ba = i, ar
        if best < 0:
            break
        ent = ent[:best] + kids(ent[best]) + ent[best + 1:]
    return ent


def _leaf_range(c, a, esc, L0, memo):
    """[first, last] leaf of node c (leaves are in sorted order left to right)."""
    if c >= L0:
        return c - L0, c - L0
    if c not in memo:
        L = a[c]
        memo[c] = (_leaf_range(L, a, esc, L0, memo)[0], _leaf_range(esc[L], a, esc, L0, memo)[1])
    return memo[c]


def _check_wide(R, tris, arity=4):
    tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
    n = len(tris)
    R.config_set("build.wide_arity", arity)
    try:
        with R.Scene.from_soup(tris) as s:
            s.build()
            assert s.wide_arity == arity
            nodes = s.read_bvh()["nodes"]
            rec = s.read_wide()
    finally:
        R.config_set("build.wide_arity", 4)
    assert rec.shape == (n - 1, 24 if arity == 8 else 16)
    L0 = n - 1
    a, esc = nodes["a"].astype(np.int64), nodes["esc"].astype(np.int64)
    lo_e, hi_e = nodes["lo"], nodes["hi"]
    lo_q, hi_q = _decode_planes(rec)
    W, wild, mask, refs = _layout(rec)
    assert W == arity
    memo = {}
    for X in range(n - 1):
        kids = _entries(X, a, esc, lo_e, hi_e, L0, arity)
        # a preorder cut of X's subtree: consecutive leaf ranges covering X's
        rng = [_leaf_range(c, a, esc, L0, memo) for c in kids]
        xl, xh = _leaf_range(X, a, esc, L0, memo)
        assert rng[0][0] == xl and rng[-1][1] == xh, X
        assert all(rng[i][1] + 1 == rng[i + 1][0] for i in range(len(rng) - 1)), X
        assert len(kids) == min(arity, xh - xl + 1), X
        assert mask[X] == (1 << len(kids)) - 1, X
        for i, c in enumerate(kids):
            want = c if c < L0 else (LEAF | (c - L0))
            assert refs[X, i] == want, (X, i)
            if not wild[X]:
                assert np.all(lo_q[X, :, i] <= lo_e[c]), (X, i)   # outward rounding, exactly
                assert np.all(hi_q[X, :, i] >= hi_e[c]), (X, i)
        assert np.all(refs[X, len(kids):] == SENT)
    return rec


def test_wide_records_small_and_degenerate(R, oracle):
    """K7w records (the greedy largest-surface cut) on small and degenerate
    scenes: every record is a preorder cut with outward-rounded boxes."""
    _check = lambda t: _check_wide(R, t)  # noqa: E731
    _check(oracle.soup(3000, 2).reshape(-1, 9))
    rng = np.random.default_rng(3)
    flat = oracle.soup(2000, 4).reshape(-1, 9).copy()
    flat[:, 2::3] = 0.25                                      # zero extent in z
    _check(flat)
    tiny = (rng.random((1500, 9)) * 1e-30).astype(np.float32)  # denormal-scale grids
    _check(tiny)
    huge = (rng.random((1500, 9)) * 3e37 - 1.5e37).astype(np.float32)
    _check(huge)
    _check(np.tile(oracle.soup(1, 3).reshape(-1, 9), (700, 1)))  # identical boxes
    two = oracle.soup(2, 9).reshape(-1, 9)
    rec = _check(two)
    assert rec.shape[0] == 1


@pytest.mark.parametrize("arity", [4, 8])
def test_wide_records_nonfinite_are_wild(R, oracle, arity):
    tris = oracle.soup(500, 6).reshape(-1, 9).copy()
    tris[17, 0] = np.inf
    tris[301, 4] = -np.inf
    rec = _check_wide(R, tris, arity)
    assert _layout(rec)[1].any()


def _render_all(R, tris, cam, w, h, spp, variant, cap=14):
    R.config_set("trace.variant", variant)
    R.config_set("trace.stack_cap", cap)
    with R.Scene.from_soup(tris) as s:
        s.build()
        hits, rgba, _ = s.render(cam, w, h, spp)
    return hits, rgba


def _oracle_render(oracle, tris, ocam, w, h, spp):
    exp = oracle.build(tris)
    hits, _ = oracle.trace(exp["nodes"], tris, ocam, w, h, spp)
    return hits, oracle.shade(hits, w, h, spp)


def _same(hits, rgba, eh, er):
    assert np.array_equal(hits["prim"], eh["prim"])
    for f in ("t", "u", "v"):
        assert np.array_equal(bits(hits[f]), bits(eh[f])), f
    assert np.array_equal(rgba, er)


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("cap", [1, 2, 3, 14])
def test_variants_and_stack_overflow(R, oracle, variant, cap):
    """cap 1-3 force the overflow hand-off to the binary traversal on most rays."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = oracle.soup(30000, 11).reshape(-1, 9)
    w, h, spp = 96, 64, 2
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    ocam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, er = _oracle_render(oracle, tris, ocam, w, h, spp)
    hits, rgba = _render_all(R, tris, cam, w, h, spp, variant, cap)
    _same(hits, rgba, eh, er)


@pytest.mark.parametrize("cap", [2, 14])
def test_greedy_cut_renders_identically(R, oracle, cap):
    """The greedy K7w cut gives the oracle's hits and image, with and without
    forced stack overflows."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = oracle.soup(40000, 13).reshape(-1, 9)
    w, h, spp = 120, 72, 1
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    ocam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    eh, er = _oracle_render(oracle, tris, ocam, w, h, spp)
    try:
        hits, rgba = _render_all(R, tris, cam, w, h, spp, 0, cap)
    finally:
        R.config_set("trace.stack_cap", 0)
    _same(hits, rgba, eh, er)


@pytest.mark.parametrize("variant", VARIANTS)
def test_variants_presets(R, oracle, variant):
    from gpu_raytracer_amd import scenes as S
    for tris, view, (w, h, spp) in [(S.cornell_tris(), S.CORNELL_VIEW, (64, 64, 1)),
                                    (S.bunny_substitute_tris(), S.BUNNY_VIEW, (160, 90, 1)),
                                    (S.sponza_substitute_tris(), S.SPONZA_VIEW, (96, 54, 1))]:
        tris = np.ascontiguousarray(tris, np.float32).reshape(-1, 9)
        cam = R.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        ocam = oracle.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        eh, er = _oracle_render(oracle, tris, ocam, w, h, spp)
        hits, rgba = _render_all(R, tris, cam, w, h, spp, variant)
        _same(hits, rgba, eh, er)


def _cams(R, oracle, eye, w00, du, dv):
    c = R._lib.rt_camera()
    o = oracle.Camera()
    for name, v in (("eye", eye), ("w00", w00), ("du", du), ("dv", dv)):
        arr = np.asarray(v, np.float32)
        for k in range(3):
            getattr(c, name)[k] = float(arr[k])
            getattr(o, name)[k] = float(arr[k])
    return c, o


@pytest.mark.parametrize("variant", VARIANTS)
def test_zero_direction_components(R, oracle, variant):
    """1/d infinite on an axis: the wide path hands these rays to the binary
    traversal.  Camera A: d.y == 0 for every ray; camera B: d.x == 0 exactly
    on pixel column 10 (w00.x = -10.5/64, du.x = 1/64)."""
    tris = oracle.soup(20000, 12).reshape(-1, 9)
    w, h = 64, 48
    cams = [
        _cams(R, oracle, (0.5, 0.5, -1.0), (-0.5, 0.0, 1.0), (1.0 / 64, 0.0, 0.0), (0.0, 0.0, 1.0 / 64)),
        _cams(R, oracle, (0.5, 0.5, -1.5), (-10.5 / 64, 0.4, 1.0), (1.0 / 64, 0.0, 0.0), (0.0, -1.0 / 64, 0.0)),
    ]
    for cam, ocam in cams:
        eh, er = _oracle_render(oracle, tris, ocam, w, h, 1)
        hits, rgba = _render_all(R, tris, cam, w, h, 1, variant)
        _same(hits, rgba, eh, er)
        assert (eh["prim"] != SENT).any()


def test_wide_work_counters(R, oracle):
    """The wide kernel fetches ~4x fewer node records than §9.7 visits nodes and
    loads a superset of the triangles §9.7 tests."""
    from gpu_raytracer_amd.scenes import SOUP_VIEW as V
    tris = oracle.soup(200000, 1).reshape(-1, 9)
    w, h = 320, 180
    cam = R.camera_look_at(V.eye, V.at, V.up, V.vfov, w, h)
    R.config_set("trace.variant", 0)
    R.config_set("trace.stack_cap", 0)
    with R.Scene.from_soup(tris) as s:
        s.build()
        binary = s.render_counters(cam, w, h, 1)
        wide = s.render_work(cam, w, h, 1)
    assert wide[0] * 2 < binary[0]
    assert wide[1] >= binary[1]


