"""Regenerate the committed golden fixtures under tests/golden/.

Run in the container (needs only numpy + the C oracle):  python tests/golden/make_golden.py

Parity status: UNPINNED against upstream SoslanGM/gpu_raytracer -- the
reference @ v0 holds no code, tests or vectors.  These
fixtures are produced by the independent numpy restatement
(oracle/oracle_np.py) of the SURVEY.md §9 contract, and the script refuses to
write them unless the C oracle (oracle/rt_oracle.c) reproduces every array
bit-for-bit.  tests/test_oracle.py then pins the C oracle to these files, and
the GPU parity tests pin librtamd to the C oracle.

Fixtures (numpy .npz, allow_pickle=False; SHA-256 in MANIFEST.json):
  soup1024.npz    N=1024 soup (seed 1): tris, bounds, morton keys, sorted
                  keys/vals, topology (left/right/range/parent/escape), node
                  AABBs, 64x48x1 and 32x24x3 hits + counters + RGBA.
  karras8.npz     SURVEY.md §9.8 Fig.-4 keys: topology + escape links.
  cornell.npz     32-tri Cornell box, 256x256x1 RGBA + 64x64x1 hits.
  edge.npz        degenerate inputs: n=1, n=2, 64 identical triangles.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from oracle import oracle_np as NP  # noqa: E402
from gpu_raytracer_amd.scenes import CORNELL_VIEW, SOUP_VIEW, cornell_tris  # noqa: E402


def u32(a):
    return np.ascontiguousarray(a).view(np.uint32)


def same(a, b, what):
    a = np.asarray(a)
    b = np.asarray(b)
    if a.dtype.kind == "f":
        a = u32(a.astype(np.float32))
    if b.dtype.kind == "f":
        b = u32(b.astype(np.float32))
    if a.shape != b.shape or not np.array_equal(a, b):
        raise SystemExit(f"C oracle and numpy restatement disagree on {what}")


def scene_arrays(prefix, tris, view, renders):
    """Build + renders via numpy; cross-check each array against the C oracle."""
    out = {}
    n = len(tris)
    b = NP.build(tris)
    c = O.build(tris)
    same(b["blo"], c["lo"], "bounds lo"); same(b["bhi"], c["hi"], "bounds hi"); same(b["inv"], c["inv"], "inv")
    same(b["skeys"], c["keys"], "sorted keys"); same(b["svals"], c["vals"], "sorted vals")
    same(b["parent"], c["parent"], "parent")
    same(b["lo"], c["nodes"]["lo"], "node lo"); same(b["hi"], c["nodes"]["hi"], "node hi")
    same(b["a"], c["nodes"]["a"], "node a"); same(b["esc"], c["nodes"]["esc"], "node esc")
    kc, vc = O.morton(tris, c["lo"], c["inv"])
    same(b["keys"], kc, "morton keys")
    out.update({f"{prefix}tris": tris, f"{prefix}bounds": np.concatenate([b["blo"], b["bhi"], b["inv"]]),
                f"{prefix}keys": b["keys"], f"{prefix}skeys": b["skeys"], f"{prefix}svals": b["svals"],
                f"{prefix}left": b["left"], f"{prefix}right": b["right"], f"{prefix}rlo": b["rlo"],
                f"{prefix}rhi": b["rhi"], f"{prefix}parent": b["parent"], f"{prefix}esc": b["esc"],
                f"{prefix}node_lo": b["lo"], f"{prefix}node_hi": b["hi"], f"{prefix}node_a": b["a"]})
    for (w, h, spp, with_hits) in renders:
        camn = NP.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        camc = O.camera_look_at(view.eye, view.at, view.up, view.vfov, w, h)
        same(camn, camc.as_array(), "camera")
        tb, hu, hv, hp, nn, nt = NP.trace(b, tris, camn, w, h, spp)
        hc, cc = O.trace(c["nodes"], tris, camc, w, h, spp, nthreads=4)
        same(tb, hc["t"], "hit t"); same(hu, hc["u"], "hit u"); same(hv, hc["v"], "hit v")
        same(hp, hc["prim"], "hit prim")
        if not (int(nn.sum()) == int(cc[0]) and int(nt.sum()) == int(cc[1])):
            raise SystemExit("counters disagree")
        rgba = NP.shade(tb, hu, hv, hp, w, h, spp)
        same(rgba, O.shade(hc, w, h, spp), "rgba")
        tag = f"{prefix}r{w}x{h}x{spp}_"
        out[tag + "cam"] = camn
        out[tag + "rgba"] = rgba
        out[tag + "counters"] = np.array([nn.sum(), nt.sum()], np.uint64)
        if with_hits:
            out[tag + "t"] = tb; out[tag + "u"] = hu; out[tag + "v"] = hv; out[tag + "prim"] = hp
    return out


def main():
    O.build_oracle()
    files = {}
    # soup N=1024
    tris = NP.soup(1024, 1)
    same(tris, O.soup(1024, 1), "soup generator")
    files["soup1024.npz"] = scene_arrays("", tris, SOUP_VIEW, [(64, 48, 1, True), (32, 24, 3, True)])
    # Karras Fig. 4
    keys = np.array([1, 2, 4, 5, 19, 24, 25, 30], np.uint32)
    l, r, rlo, rhi, par = NP.karras(keys)
    esc = NP.escape(8, l, r, par)
    lc, rc, rloc, rhic, parc = O.karras(keys)
    same(l, lc, "karras left"); same(r, rc, "karras right"); same(par, parc, "karras parent")
    same(esc, O.escape(8, lc, rc, parc), "karras esc")
    files["karras8.npz"] = dict(keys=keys, left=l, right=r, rlo=rlo, rhi=rhi, parent=par, esc=esc)
    # Cornell
    ct = cornell_tris()
    files["cornell.npz"] = scene_arrays("", ct, CORNELL_VIEW, [(256, 256, 1, False), (64, 64, 1, True)])
    # edge cases
    edge = {}
    edge.update(scene_arrays("n1_", NP.soup(1, 7), SOUP_VIEW, [(16, 16, 2, True)]))
    edge.update(scene_arrays("n2_", NP.soup(2, 7), SOUP_VIEW, [(16, 16, 1, True)]))
    same_tri = np.tile(NP.soup(1, 3), (64, 1))
    edge.update(scene_arrays("dup64_", same_tri, SOUP_VIEW, [(16, 16, 1, True)]))
    files["edge.npz"] = edge

    manifest = {}
    for name, arrays in files.items():
        path = os.path.join(HERE, name)
        np.savez_compressed(path, **arrays)
        manifest[name] = hashlib.sha256(open(path, "rb").read()).hexdigest()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=2, sort_keys=True)
        f.write("\n")
    print(json.dumps(manifest, indent=2))


if __name__ == "__main__":
    main()
