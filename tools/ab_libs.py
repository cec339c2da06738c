"""A/B of librtamd builds: alternating measurement processes (tools/ab_child.py,
one library per process via RT_LIB), medians per library, and a check that
every library produced identical outputs.
usage: python tools/ab_libs.py ROUNDS MODES lib1.so lib2.so ...
A library argument may carry a config: lib.so@trace.steal=1 (RT_CONFIG)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rounds, modes, libs = int(sys.argv[1]), sys.argv[2], sys.argv[3:]
res = {lib: [] for lib in libs}
for r in range(rounds):
    for lib in libs:
        path, _, cfg = lib.partition("@")
        env = dict(os.environ, RT_LIB=os.path.abspath(path), RT_CONFIG=cfg)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "ab_child.py"), modes], env=env,
                           capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stdout, p.stderr)
            sys.exit(p.returncode)
        res[lib].append(json.loads(p.stdout.strip().splitlines()[-1]))
        print(r, os.path.basename(lib), res[lib][-1], flush=True)
keys = [k for k in res[libs[0]][0] if not k.startswith("crc")]
for lib in libs:
    print(f"{os.path.basename(lib):<28s}", "  ".join(f"{k} {np.median([x[k] for x in res[lib]]):.4f}" for k in keys))
crcs = {lib: {k: v for k, v in res[lib][0].items() if k.startswith("crc")} for lib in libs}
same = all(c == crcs[libs[0]] for c in crcs.values())
print("outputs identical across libraries:", same, crcs[libs[0]])
