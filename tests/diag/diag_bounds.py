"""(tests/diag: uses the oracle as the checker.) Diagnostic: rt_stage_bounds vs oracle over many n (prints mismatches)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import gpu_raytracer_amd as R
from oracle import oracle as O
for n in [1, 2, 3, 7, 63, 64, 65, 128, 255, 256, 257, 511, 512, 513, 1000, 4096, 5000]:
    t = O.soup(n, 4).reshape(-1, 9)
    lo, hi, inv = R.stage_bounds(t)
    elo, ehi, einv = O.centroid_bounds(t)
    ok = np.array_equal(lo.view(np.uint32), elo.view(np.uint32)) and np.array_equal(hi.view(np.uint32), ehi.view(np.uint32)) and np.array_equal(inv.view(np.uint32), einv.view(np.uint32))
    print(n, "OK" if ok else f"BAD lo={lo} hi={hi} inv={inv} exp lo={elo} hi={ehi} inv={einv}", flush=True)
