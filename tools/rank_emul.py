"""bench.py's rank_emulation for one BASELINE config, standalone (the same
function the bench line runs), with librtamd knobs: one GPU plays each rank
of a P-GPU run in turn on the bench's orbiting camera.  Prints the JSON
block.  Under `rocprofv3 --kernel-trace` it gives the per-rank kernel trace.
usage: python tools/rank_emul.py [config=5] [frames=6] [ranks=2,4,8] [knob=value ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import gpu_raytracer_amd as R  # noqa: E402
from gpu_raytracer_amd import scenes as S  # noqa: E402

args = dict(a.split("=", 1) for a in sys.argv[1:])
key = int(args.pop("config", 5))
frames = int(args.pop("frames", 6))
ranks = tuple(int(x) for x in args.pop("ranks", "2,4,8").split(","))
for k, v in args.items():
    R.config_set(k, int(v))
    print(f"{k} = {v}", file=sys.stderr, flush=True)
dev = torch.device("cuda", 0)
cfg = S.CONFIGS[key]
scene = bench.make_scene(R, S, cfg)
scene.build()
out = bench.rank_emulation(R, S, scene, key, torch, dev, frames=frames, ranks=ranks)
out["knobs"] = args
print(json.dumps(out), flush=True)
scene.close()
