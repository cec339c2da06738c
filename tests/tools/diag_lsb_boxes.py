"""Diagnostic: which node boxes differ from the oracle after an LSB-sorted
build (build.sort = 0) of the 1M soup -- local or crossing nodes, and the
range lengths / block positions of the bad ones.  RT_LIB selects a library.
usage: python tests/tools/diag_lsb_boxes.py [n] [refit_leaves]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import gpu_raytracer_amd as R  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 512
tris = O.soup(n, 77).reshape(-1, 9)
exp = O.build(tris)
left, right, rlo, rhi, parent = O.karras(exp["keys"])
for sort in (2, 0):
    R.config_set("build.sort", sort)
    with R.Scene.from_soup(tris) as s:
        s.build()
        s.build()
        got = s.read_bvh()
        t = s.build_times()
    g, e = got["nodes"], exp["nodes"]
    bad = np.nonzero(np.any(g["lo"][: n - 1].view(np.uint32) != e["lo"][: n - 1].view(np.uint32), axis=1)
                     | np.any(g["hi"][: n - 1].view(np.uint32) != e["hi"][: n - 1].view(np.uint32), axis=1))[0]
    print(f"sort={sort} kind={t.sort_kind} keys_ok={np.array_equal(got['keys'], exp['keys'])} "
          f"topo_ok={np.array_equal(g['a'], e['a']) and np.array_equal(g['esc'], e['esc'])} bad internal boxes={bad.size}")
    if bad.size:
        lo, hi = rlo[bad], rhi[bad]
        cross = (lo // T) != (hi // T)
        print(f"  crossing {int(cross.sum())} local {int((~cross).sum())}; range len min {int((hi - lo).min()) + 1} "
              f"max {int((hi - lo).max()) + 1}; first {bad[:10].tolist()}")
        for i in bad[:5]:
            print(f"  node {i}: range [{rlo[i]}, {rhi[i]}] blocks {rlo[i] // T}..{rhi[i] // T} got lo "
                  f"{g['lo'][i].tolist()} exp {e['lo'][i].tolist()}")
R.config_set("build.sort", 2)
