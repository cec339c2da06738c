"""CPU tests of the oracle itself (test infrastructure): known answers from
SURVEY.md §4/§9.8, the committed golden fixtures, and the independent numpy
restatement.  Parity vs upstream SoslanGM/gpu_raytracer is unpinned (the
reference holds no code or vectors); these tests pin the oracle
to the contract and to its second, independent restatement."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, bits, load_golden

SENT = 0xFFFFFFFF


def test_manifest_hashes():
    man = json.load(open(os.path.join(GOLDEN, "MANIFEST.json")))
    assert set(man) == {"soup1024.npz", "karras8.npz", "cornell.npz", "edge.npz"}
    for name, h in man.items():
        assert hashlib.sha256(open(os.path.join(GOLDEN, name), "rb").read()).hexdigest() == h, name


def test_morton_kat(oracle):
    L = oracle.lib()
    assert L.orc_expand10(1023) == 0x09249249
    assert L.orc_morton3(1023, 1023, 1023) == 0x3FFFFFFF
    assert L.orc_morton3(1, 0, 0) == 0x4
    assert L.orc_morton3(0, 1, 0) == 0x2
    assert L.orc_morton3(0, 0, 1) == 0x1
    assert L.orc_expand10(0) == 0


def test_karras_fig4_kat(oracle):
    """Karras 2012 Fig. 4 keys {1,2,4,5,19,24,25,30}."""
    keys = np.array([1, 2, 4, 5, 19, 24, 25, 30], np.uint32)
    left, right, rlo, rhi, parent = oracle.karras(keys)
    I = lambda i: i
    Lf = lambda k: 7 + k
    exp = {  # node: (range, left, right, esc)
        0: ((0, 7), I(3), I(4), SENT), 1: ((0, 1), Lf(0), Lf(1), I(2)), 2: ((2, 3), Lf(2), Lf(3), I(4)),
        3: ((0, 3), I(1), I(2), I(4)), 4: ((4, 7), Lf(4), I(5), SENT), 5: ((5, 7), I(6), Lf(7), SENT),
        6: ((5, 6), Lf(5), Lf(6), Lf(7)),
    }
    esc = oracle.escape(8, left, right, parent)
    for i, (rng, l, r, e) in exp.items():
        assert (rlo[i], rhi[i]) == rng, i
        assert left[i] == l and right[i] == r and esc[i] == e, i
    leaf_esc = [Lf(1), I(2), Lf(3), I(4), I(5), Lf(6), Lf(7), SENT]
    assert list(esc[7:]) == leaf_esc
    g = load_golden("karras8.npz")
    for k in ("left", "right", "rlo", "rhi", "parent", "esc"):
        ref = {"left": left, "right": right, "rlo": rlo, "rhi": rhi, "parent": parent, "esc": esc}[k]
        assert np.array_equal(g[k], ref), k


def test_mt_kat(oracle):
    tri = [-1, -1, 0, 1, -1, 0, -1, 1, 0]
    hit, t, u, v = oracle.intersect_tri([0, 0, -1], [0, 0, 1], tri)
    assert hit and (t, u, v) == (1.0, 0.5, 0.5)
    # (0,0) lies on the hypotenuse: u + v == 1 exactly and is accepted (no epsilon)
    assert u + v == 1.0
    assert not oracle.intersect_tri([0.5, 0.5, -1], [0, 0, 1], tri)[0]  # outside: u + v > 1
    # parallel ray: det == 0 -> miss; behind origin: t <= 0 -> miss; t_best cull (strict <)
    assert not oracle.intersect_tri([0, 0, -1], [1, 0, 0], tri)[0]
    assert not oracle.intersect_tri([0, 0, 1], [0, 0, 1], tri)[0]
    assert not oracle.intersect_tri([0, 0, -1], [0, 0, 1], tri, t_best=1.0)[0]
    assert oracle.intersect_tri([0, 0, -1], [0, 0, 1], tri, t_best=np.nextafter(np.float32(1), np.float32(2)))[0]


def test_minmax_semantics(oracle):
    L = oracle.lib()
    assert np.signbit(L.orc_fmin(-0.0, 0.0)) and np.signbit(L.orc_fmin(0.0, -0.0))
    assert not np.signbit(L.orc_fmax(-0.0, 0.0)) and not np.signbit(L.orc_fmax(0.0, -0.0))
    assert L.orc_fmin(float("nan"), 2.0) == 2.0 and L.orc_fmin(2.0, float("nan")) == 2.0
    assert L.orc_fmax(float("nan"), -2.0) == -2.0
    assert L.orc_fmin(float("inf"), 3.0) == 3.0


def test_pcg_hash(oracle):
    def ref(x):
        m = 0xFFFFFFFF
        st = (x * 747796405 + 2891336453) & m
        w = (((st >> ((st >> 28) + 4)) ^ st) * 277803737) & m
        return ((w >> 22) ^ w) & m
    for x in [0, 1, 2, 12345, 0xFFFFFFFF, 2073599, 987654321]:
        assert oracle.lib().orc_pcg_hash(x) == ref(x)


@pytest.mark.parametrize("kind", ["random", "equal", "sorted", "reversed", "onebucket", "hibits"])
def test_sort_equals_stable_sort(oracle, kind):
    rng = np.random.default_rng(5)
    n = 20000
    keys = {
        "random": rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
        "equal": np.full(n, 0xDEADBEEF, np.uint32),
        "sorted": np.arange(n, dtype=np.uint32) * 3,
        "reversed": (np.arange(n, dtype=np.uint32)[::-1] * 7).copy(),
        "onebucket": (rng.integers(0, 256, n) << 8).astype(np.uint32),
        "hibits": (rng.integers(0, 4, n).astype(np.uint32) << 30),
    }[kind]
    vals = np.arange(n, dtype=np.uint32)
    k, v = oracle.radix_sort(keys, vals)
    o = np.argsort(keys, kind="stable")
    assert np.array_equal(k, keys[o]) and np.array_equal(v, vals[o])


def _check_scene(oracle, g, prefix=""):
    tris = g[prefix + "tris"]
    b = oracle.build(tris)
    assert np.array_equal(bits(b["lo"]), bits(g[prefix + "bounds"][0:3]))
    assert np.array_equal(bits(b["hi"]), bits(g[prefix + "bounds"][3:6]))
    assert np.array_equal(bits(b["inv"]), bits(g[prefix + "bounds"][6:9]))
    keys, vals = oracle.morton(tris, b["lo"], b["inv"])
    assert np.array_equal(keys, g[prefix + "keys"])
    assert np.array_equal(b["keys"], g[prefix + "skeys"]) and np.array_equal(b["vals"], g[prefix + "svals"])
    assert np.array_equal(b["parent"], g[prefix + "parent"])
    nd = b["nodes"]
    assert np.array_equal(bits(nd["lo"]), bits(g[prefix + "node_lo"]))
    assert np.array_equal(bits(nd["hi"]), bits(g[prefix + "node_hi"]))
    assert np.array_equal(nd["a"], g[prefix + "node_a"]) and np.array_equal(nd["esc"], g[prefix + "esc"])
    for key in [k for k in g if k.startswith(prefix + "r") and k.endswith("_cam")]:
        tag = key[: -len("cam")]
        w, h, spp = (int(x) for x in tag[len(prefix) + 1: -1].split("x"))
        cam = oracle.Camera()
        c = g[key]
        for i, f in enumerate(("eye", "w00", "du", "dv")):
            getattr(cam, f)[:] = [float(x) for x in c[i]]
        hits, cnt = oracle.trace(nd, tris, cam, w, h, spp, nthreads=4)
        assert cnt[0] == g[tag + "counters"][0] and cnt[1] == g[tag + "counters"][1]
        assert np.array_equal(oracle.shade(hits, w, h, spp), g[tag + "rgba"])
        if tag + "t" in g:
            assert np.array_equal(bits(hits["t"]), bits(g[tag + "t"]))
            assert np.array_equal(bits(hits["u"]), bits(g[tag + "u"]))
            assert np.array_equal(bits(hits["v"]), bits(g[tag + "v"]))
            assert np.array_equal(hits["prim"], g[tag + "prim"])


def test_golden_soup1024(oracle):
    g = load_golden("soup1024.npz")
    assert np.array_equal(bits(oracle.soup(1024, 1)), bits(g["tris"]))
    _check_scene(oracle, g)


def test_golden_cornell(oracle):
    from gpu_raytracer_amd.scenes import CORNELL_VIEW, cornell_tris
    g = load_golden("cornell.npz")
    assert np.array_equal(bits(cornell_tris()), bits(g["tris"]))
    cam = oracle.camera_look_at(CORNELL_VIEW.eye, CORNELL_VIEW.at, CORNELL_VIEW.up, CORNELL_VIEW.vfov, 256, 256)
    assert np.array_equal(bits(cam.as_array()), bits(g["r256x256x1_cam"]))
    _check_scene(oracle, g)


def test_golden_edge(oracle):
    g = load_golden("edge.npz")
    for p in ("n1_", "n2_", "dup64_"):
        _check_scene(oracle, g, p)


@pytest.mark.parametrize("n", [3, 5, 17, 300, 2049])
def test_oracle_vs_numpy_restatement(oracle, n):
    from oracle import oracle_np as NP
    tris = NP.soup(n, 11)
    assert np.array_equal(bits(tris), bits(oracle.soup(n, 11)))
    b = oracle.build(tris)
    bn = NP.build(tris)
    assert np.array_equal(b["keys"], bn["skeys"]) and np.array_equal(b["vals"], bn["svals"])
    assert np.array_equal(bits(b["nodes"]["lo"]), bits(bn["lo"]))
    assert np.array_equal(bits(b["nodes"]["hi"]), bits(bn["hi"]))
    assert np.array_equal(b["nodes"]["esc"], bn["esc"]) and np.array_equal(b["nodes"]["a"], bn["a"])
    cam = oracle.camera_look_at([0.5, 0.5, -1.5], [0.5, 0.5, 0.5], [0, 1, 0], 45, 24, 16)
    hits, cnt = oracle.trace(b["nodes"], tris, cam, 24, 16, 2, nthreads=2)
    tb, hu, hv, hp, nn, nt = NP.trace(bn, tris, cam.as_array(), 24, 16, 2)
    assert np.array_equal(bits(hits["t"]), bits(tb)) and np.array_equal(hits["prim"], hp)
    assert cnt[0] == nn.sum() and cnt[1] == nt.sum()


def test_trace_row_sampling_and_threads(oracle):
    """Row-subsampled, multi-threaded trace == the same rows of a full trace."""
    tris = oracle.soup(4000, 2)
    b = oracle.build(tris)
    cam = oracle.camera_look_at([0.5, 0.5, -1.5], [0.5, 0.5, 0.5], [0, 1, 0], 45, 40, 30)
    full, c_full = oracle.trace(b["nodes"], tris, cam, 40, 30, 1, nthreads=1)
    sub, c_sub = oracle.trace(b["nodes"], tris, cam, 40, 30, 1, row0=1, row_step=3, nthreads=3)
    f = full.reshape(30, 40)
    s = sub.reshape(30, 40)
    assert np.array_equal(bits(f["t"][1::3]), bits(s["t"][1::3]))
    assert c_sub[0] < c_full[0]


def test_trace_survives_failed_thread_creation(oracle):
    """A worker thread that cannot be created (EAGAIN under the GPU box's task
    cap) must not leave pixels at the initial "miss": the calling thread
    drains the trace's shared cursor and runs a path job's rows itself.  Before
    r03 the creation status was ignored and glibc's pthread_join of the unset
    id returns ESRCH at once -- with every creation failing the expected hits
    were all misses (DESIGN.md "The r02 8-ary wrong-hit record")."""
    from gpu_raytracer_amd import scenes as S
    tris = np.ascontiguousarray(S.cornell_tris(), np.float32).reshape(-1, 9)
    V, light = S.CORNELL_VIEW, S.LIGHTS["cornell"]
    cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, 64, 64)
    b = oracle.build(tris)
    ref, cref = oracle.trace(b["nodes"], tris, cam, 64, 64, 1, nthreads=1)
    _, pref, pcref = oracle.render_path(b["nodes"], tris, cam, 32, 32, 2, light, 0.2, 2, nthreads=1)
    lib = oracle.lib()
    lib.orc_debug_fail_spawn(1)
    try:
        got, cgot = oracle.trace(b["nodes"], tris, cam, 64, 64, 1, nthreads=8)
        _, pgot, pcgot = oracle.render_path(b["nodes"], tris, cam, 32, 32, 2, light, 0.2, 2, nthreads=8)
    finally:
        lib.orc_debug_fail_spawn(0)
    assert (ref["prim"] != 0xFFFFFFFF).sum() > 1000
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)) and np.array_equal(cgot, cref)
    assert np.array_equal(pgot, pref) and np.array_equal(pcgot, pcref)


def _secondary_scenes(oracle):
    from gpu_raytracer_amd import scenes as S
    return [(np.ascontiguousarray(S.cornell_tris(), np.float32).reshape(-1, 9), S.CORNELL_VIEW, S.LIGHTS["cornell"], 24),
            (oracle.soup(3000, 41).reshape(-1, 9), S.SOUP_VIEW, S.LIGHTS["soup"], 24)]


def test_shadow_oracle_vs_numpy_restatement(oracle):
    """Shadow mode: the C oracle and the independent wavefront
    numpy restatement agree bit for bit."""
    from oracle import oracle_np as NP
    for tris, V, light, w in _secondary_scenes(oracle):
        cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, w)
        b = oracle.build(tris)
        eh, er, _ = oracle.render_shadow(b["nodes"], tris, cam, w, w, 2, light, 0.2)
        t, u, v, p, rgba = NP.render_shadow(NP.build(tris), tris, cam.as_array(), w, w, 2, light, 0.2)
        assert np.array_equal(eh["prim"], p) and np.array_equal(bits(eh["t"]), bits(t))
        assert np.array_equal(er, rgba)


@pytest.mark.parametrize("depth", [0, 1, 3])
def test_path_oracle_vs_numpy_restatement(oracle, depth):
    """Path mode: the C oracle (per-pixel recursion) and the numpy
    restatement (a wavefront over all live paths) agree bit for bit, ray
    count included."""
    from oracle import oracle_np as NP
    for tris, V, light, w in _secondary_scenes(oracle):
        cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, w, w)
        b = oracle.build(tris)
        eh, er, cnt = oracle.render_path(b["nodes"], tris, cam, w, w, 2, light, 0.3, depth, nthreads=3)
        t, u, v, p, rgba, nrays = NP.render_path(NP.build(tris), tris, cam.as_array(), w, w, 2, light, 0.3, depth)
        assert np.array_equal(eh["prim"], p) and np.array_equal(bits(eh["t"]), bits(t))
        assert np.array_equal(er, rgba)
        assert int(cnt[2]) == nrays
        assert nrays > w * w * 2


def test_path_oracle_properties(oracle):
    """Thread-count independence; more sky or more bounces never darkens a
    pixel (every term is non-negative); depth 0 ignores the sky."""
    from gpu_raytracer_amd import scenes as S
    tris = np.ascontiguousarray(S.cornell_tris(), np.float32).reshape(-1, 9)
    V, light = S.CORNELL_VIEW, S.LIGHTS["cornell"]
    cam = oracle.camera_look_at(V.eye, V.at, V.up, V.vfov, 40, 40)
    b = oracle.build(tris)
    _, a1, c1 = oracle.render_path(b["nodes"], tris, cam, 40, 40, 2, light, 0.2, 2, nthreads=1)
    _, a4, c4 = oracle.render_path(b["nodes"], tris, cam, 40, 40, 2, light, 0.2, 2, nthreads=4)
    assert np.array_equal(a1, a4) and np.array_equal(c1, c4)
    _, dark, _ = oracle.render_path(b["nodes"], tris, cam, 40, 40, 2, light, 0.0, 2)
    _, bright, _ = oracle.render_path(b["nodes"], tris, cam, 40, 40, 2, light, 1.0, 2)
    assert (bright >= dark).all() and (bright > dark).any()
    _, d0a, _ = oracle.render_path(b["nodes"], tris, cam, 40, 40, 2, light, 0.0, 0)
    _, d0b, _ = oracle.render_path(b["nodes"], tris, cam, 40, 40, 2, light, 1.0, 0)
    assert np.array_equal(d0a, d0b)
    assert (dark >= d0a).all()
