"""How much would the refit's triangle gather gain from a tile-bucketed copy
of the soup?  k_topo_refit reads each sorted leaf's
36-B triangle at its ORIGINAL index (vals[i]): random lines over the whole
soup.  K1 could instead write the triangles of each 4096-prim sort tile
grouped by top-10-bit bucket -- the layout its key words already have -- and
the gather sort hand the refit each leaf's position in that copy.  This
measures the two read patterns alone, with torch's index_select standing in
for the refit's gather (same rows, same order, coalesced output), after an
eviction of L2 and the Infinity Cache:
  orig      rows vals[i] of the soup (the refit today)
  bucketed  rows pos[vals[i]] of the bucketed copy
  seq       rows i (the streaming floor)
The copy's in-bucket order is index order (K1's is the LDS atomics'; the
sort scatters a run's prims over its bucket either way).
usage: python tools/gather_layout.py [n=10000000] [reps=20]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
s = R.Scene.generate_soup(n, 1)
s.build()
b = s.read_bvh()
keys, vals = b["keys"], b["vals"]
tris = np.ascontiguousarray(s.tris(), np.float32).reshape(-1, 9)
s.close()
korig = np.empty(n, np.uint32)
korig[vals] = keys
prim = np.arange(n, dtype=np.int64)
order = np.lexsort((prim, korig >> 20, prim // 4096))  # tile, then bucket, then index
pos = np.empty(n, np.int64)
pos[order] = prim
dev = torch.device("cuda")
T = torch.from_numpy(tris).to(dev)
Cb = torch.from_numpy(np.ascontiguousarray(tris[order])).to(dev)
idx = {"orig": torch.from_numpy(vals.astype(np.int64)).to(dev),
       "bucketed": torch.from_numpy(pos[vals]).to(dev),
       "seq": torch.arange(n, dtype=torch.int64, device=dev)}
src = {"orig": T, "bucketed": Cb, "seq": T}
assert torch.equal(torch.index_select(Cb, 0, idx["bucketed"]), torch.index_select(T, 0, idx["orig"]))
flush = torch.empty(1 << 28, dtype=torch.int32, device=dev)  # 1 GiB: past L2 and the 256-MB Infinity Cache
out = torch.empty((n, 9), dtype=torch.float32, device=dev)
res = {k: [] for k in idx}
for _ in range(reps):
    for k in idx:
        flush.fill_(1)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.index_select(src[k], 0, idx[k], out=out)
        e.record()
        torch.cuda.synchronize()
        res[k].append(a.elapsed_time(e) * 1e3)
# lines of 128 B each pattern touches per prim, from the addresses alone (no cache)
for k in idx:
    ii = idx[k].cpu().numpy()
    first, last = (ii * 36) // 128, (ii * 36 + 35) // 128
    print(f"{k:9s} n={n} median {np.median(res[k]):8.1f} us  (min {min(res[k]):.1f})  "
          f"distinct 128-B lines per prim in 256-leaf blocks "
          f"{np.mean([len(np.unique(np.concatenate([first[j:j + 256], last[j:j + 256]]))) for j in range(0, n, 256 * 97)]) / 256 * 128:.1f} B",
          flush=True)
