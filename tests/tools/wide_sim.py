"""Step counts of the wide traversal for K-ary greedy cuts (CPU model,
tests/tools/wide_sim.c): how much an 8-wide record would shorten the heavy rays'
dependent chains.  Design experiment; uses the oracle's build.

    python tests/tools/wide_sim.py [n] [K ...]
"""
import ctypes as C
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ks = [k for k in sys.argv[2:]] or ["4", "8"]  # K, or K:sah:ci:cl (SAH-optimal cut)
    so = "/tmp/libwsim.so"
    O.lib()
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tests/tools/wide_sim.c"),
                    "-L", os.path.join(ROOT, "oracle/build"), "-loracle", "-lm",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle/build")], check=True)
    L = C.CDLL(so)
    tris = O.soup(n, 1)
    b = O.build(tris)
    nodes = b["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    ref, _ = O.trace(nodes, tris, cam, W, H)
    P = C.c_void_p
    for ks_ in ks:
        f = ks_.split(":")
        K = int(f[0])
        cut = np.empty((n - 1) * K, np.uint32)
        if len(f) > 1 and f[1] == "sah":
            L.wsim_cut_sah(nodes.ctypes.data_as(P), n, K, C.c_float(float(f[2])), C.c_float(float(f[3])),
                           cut.ctypes.data_as(P))
        else:
            L.wsim_cut(nodes.ctypes.data_as(P), n, K, cut.ctypes.data_as(P))
        steps = np.zeros(W * H, np.uint16)
        recs = np.zeros(W * H, np.uint16)
        leaves = np.zeros(W * H, np.uint16)
        hitp = np.zeros(W * H, np.uint32)
        msp = np.zeros(W * H, np.uint8)

        def band(y0):
            L.wsim_trace(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), cut.ctypes.data_as(P), K,
                         C.byref(cam), W, H, y0, min(H, y0 + 36), steps.ctypes.data_as(P),
                         recs.ctypes.data_as(P), leaves.ctypes.data_as(P), hitp.ctypes.data_as(P), msp.ctypes.data_as(P))

        with ThreadPoolExecutor(8) as ex:
            list(ex.map(band, range(0, H, 36)))
        assert np.array_equal(hitp, ref["prim"]), "model disagrees with the oracle"
        s = steps.astype(np.int64)
        # per 8x8 quadrant: the wave's steps = its slowest lane's
        q = s.reshape(H // 8, 8, W // 8, 8).max(axis=(1, 3))
        print(f"K={ks_}: records {int(recs.sum()):,} leaves {int(leaves.sum()):,} steps {int(s.sum()):,} | "
              f"per ray mean {s.mean():.2f} p99 {np.percentile(s, 99):.0f} p99.9 {np.percentile(s, 99.9):.0f} "
              f"max {s.max()} | wave(8x8) max-lane steps mean {q.mean():.1f} p99 {np.percentile(q, 99):.0f} "
              f"max {q.max()} | rays > 96 steps {(s > 96).sum()}, > 64 {(s > 64).sum()}, > 48 {(s > 48).sum()}",
              flush=True)
        print("   stack depth: " + " ".join(f">{c}:{int((msp > c).sum())}" for c in (8, 10, 12, 14, 16, 20, 24, 28)) + f" max {msp.max()}", flush=True)




def waves(n=1_000_000, policies=((0, 0), (4, 16), (4, 24), (4, 32), (6, 24), (8, 24))):
    """Wave model of leaf deferral (wsim_waves): steps, block counts, VALU."""
    so = "/tmp/libwsim.so"
    O.lib()
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tests/tools/wide_sim.c"),
                    "-L", os.path.join(ROOT, "oracle/build"), "-loracle", "-lm",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle/build")], check=True)
    L = C.CDLL(so)
    tris = O.soup(n, 1)
    b = O.build(tris)
    nodes = b["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    ref, _ = O.trace(nodes, tris, cam, W, H)
    P = C.c_void_p
    K = 4
    cut = np.empty((n - 1) * K, np.uint32)
    L.wsim_cut(nodes.ctypes.data_as(P), n, K, cut.ctypes.data_as(P))
    for F, T in policies:
        hitp = np.zeros(W * H, np.uint32)
        outs = [np.zeros(6) for _ in range(8)]
        bands = np.array_split(np.arange(H // 8), 8)

        def run(i):
            L.wsim_waves(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), cut.ctypes.data_as(P), K, C.byref(cam),
                         W, H, int(bands[i][0]), int(bands[i][-1] + 1), F, T, outs[i].ctypes.data_as(P),
                         hitp.ctypes.data_as(P))

        with ThreadPoolExecutor(8) as ex:
            list(ex.map(run, range(8)))
        o = sum(outs)
        assert np.array_equal(hitp, ref["prim"]), "model disagrees with the oracle"
        print(f"F={F} T={T}: wave-steps {o[0]:,.0f} leaf blocks {o[1]:,.0f} ({o[3] / max(o[1], 1):.1f} lanes) "
              f"record blocks {o[2]:,.0f} ({o[4] / max(o[2], 1):.1f} lanes) lane-records {o[4]:,.0f} "
              f"VALU model {o[5]:,.0f}", flush=True)


def compact(n=1_000_000, policies=((0, 0), (16, 8), (24, 8), (32, 8), (24, 16), (32, 16), (40, 16))):
    """Wave-compaction model (wsim_compact): pass 1 until < A lanes live, pass 2 packed."""
    so = "/tmp/libwsim.so"
    O.lib()
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tests/tools/wide_sim.c"),
                    "-L", os.path.join(ROOT, "oracle/build"), "-loracle", "-lm",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle/build")], check=True)
    L = C.CDLL(so)
    tris = O.soup(n, 1)
    b = O.build(tris)
    nodes = b["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    ref, _ = O.trace(nodes, tris, cam, W, H)
    P = C.c_void_p
    K = 4
    cut = np.empty((n - 1) * K, np.uint32)
    L.wsim_cut(nodes.ctypes.data_as(P), n, K, cut.ctypes.data_as(P))
    for A, Smin in policies:
        hitp = np.zeros(W * H, np.uint32)
        outs = [np.zeros(7) for _ in range(8)]
        bands = np.array_split(np.arange(H // 8), 8)

        def run(i):
            L.wsim_compact(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), cut.ctypes.data_as(P), K,
                           C.byref(cam), W, H, int(bands[i][0]), int(bands[i][-1] + 1), A, Smin,
                           outs[i].ctypes.data_as(P), hitp.ctypes.data_as(P))

        with ThreadPoolExecutor(8) as ex:
            list(ex.map(run, range(8)))
        o = sum(outs)
        assert np.array_equal(hitp, ref["prim"]), "model disagrees with the oracle"
        print(f"A={A & 0xFFFF}{' empty-only' if A & 0x10000 else ''} S={Smin}: wave-steps {o[0]:,.0f} leaf blocks {o[1]:,.0f} ({o[3] / max(o[1], 1):.1f} lanes) "
              f"record blocks {o[2]:,.0f} ({o[4] / max(o[2], 1):.1f} lanes) queued {o[6]:,.0f} "
              f"VALU model {o[5]:,.0f}", flush=True)


def chain(n=1_000_000, K=4):
    """Top-of-stack prefetch model (wsim_chain): steps whose data would already be there."""
    so = "/tmp/libwsim.so"
    O.lib()
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tests/tools/wide_sim.c"),
                    "-L", os.path.join(ROOT, "oracle/build"), "-loracle", "-lm",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle/build")], check=True)
    L = C.CDLL(so)
    tris = O.soup(n, 1)
    nodes = O.build(tris)["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    ref, _ = O.trace(nodes, tris, cam, W, H)
    P = C.c_void_p
    cut = np.empty((n - 1) * K, np.uint32)
    L.wsim_cut(nodes.ctypes.data_as(P), n, K, cut.ctypes.data_as(P))
    steps = np.zeros(W * H, np.uint16)
    ready = np.zeros(W * H, np.uint16)
    hitp = np.zeros(W * H, np.uint32)

    def band(y0):
        L.wsim_chain(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), cut.ctypes.data_as(P), K, C.byref(cam),
                     W, H, y0, min(H, y0 + 36), steps.ctypes.data_as(P), ready.ctypes.data_as(P),
                     hitp.ctypes.data_as(P))

    with ThreadPoolExecutor(8) as ex:
        list(ex.map(band, range(0, H, 36)))
    assert np.array_equal(hitp, ref["prim"]), "model disagrees with the oracle"
    s, r = steps.astype(np.int64), ready.astype(np.int64)
    print(f"K={K}: steps {s.sum():,} ready {r.sum():,} ({r.sum() / s.sum():.3f})", flush=True)
    for lo in (32, 64, 96, 128, 192):
        m = s >= lo
        if m.any():
            print(f"  rays >= {lo} steps: {int(m.sum())}, ready fraction {r[m].sum() / s[m].sum():.3f}, "
                  f"max steps {s[m].max()}, waits of the costliest {int(s[m].max() - r[m][s[m].argmax()])}", flush=True)




def merge(n=1_000_000, policies=((0, 0), (32, 8), (40, 8), (48, 8), (64, 8), (32 | 0x10000, 8), (48 | 0x10000, 8))):
    """In-block wave merging model (wsim_merge)."""
    so = "/tmp/libwsim.so"
    O.lib()
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tests/tools/wide_sim.c"),
                    "-L", os.path.join(ROOT, "oracle/build"), "-loracle", "-lm",
                    "-Wl,-rpath," + os.path.join(ROOT, "oracle/build")], check=True)
    L = C.CDLL(so)
    tris = O.soup(n, 1)
    b = O.build(tris)
    nodes = b["nodes"]
    v = S.VIEWS["soup"]
    W, H = 1920, 1080
    cam = O.camera_look_at(v.eye, v.at, v.up, v.vfov, W, H)
    ref, _ = O.trace(nodes, tris, cam, W, H)
    P = C.c_void_p
    K = 4
    cut = np.empty((n - 1) * K, np.uint32)
    L.wsim_cut(nodes.ctypes.data_as(P), n, K, cut.ctypes.data_as(P))
    for A, Smin in policies:
        hitp = np.zeros(W * H, np.uint32)
        outs = [np.zeros(7) for _ in range(8)]
        bands = np.array_split(np.arange(H // 16), 8)

        def run(i):
            L.wsim_merge(nodes.ctypes.data_as(P), n, tris.ctypes.data_as(P), cut.ctypes.data_as(P), K,
                         C.byref(cam), W, H, int(bands[i][0]), int(bands[i][-1] + 1), A, Smin,
                         outs[i].ctypes.data_as(P), hitp.ctypes.data_as(P))

        with ThreadPoolExecutor(8) as ex:
            list(ex.map(run, range(8)))
        o = sum(outs)
        mx = max(x[6] for x in outs)
        ok = np.array_equal(hitp[: (H // 16) * 16 * W], ref["prim"][: (H // 16) * 16 * W])
        print(f"A={A & 0xFFFF}{' empty-only' if A & 0x10000 else ''} S={Smin}: wave-steps {o[0]:,.0f} leaf blocks {o[1]:,.0f} record blocks {o[2]:,.0f} "
              f"VALU model {o[3]:,.0f} tile rounds sum {o[4]:,.0f} max {mx:.0f} moved {o[5]:,.0f} exact {ok}",
              flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "chain":
        chain()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "compact":
        compact()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "merge":
        merge()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "waves":
        waves()
    else:
        main()
