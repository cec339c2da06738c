#!/bin/bash
# Narrow heavy-ray groups (r06): P = 8 emulated max-rank
# time of configs[2] (soup-1M 1080p1, bench orbit) per library (RT_LIB:
# lib/exp/cg8.so, cg4.so from tools/build_exp.sh with -DRT_COOP_G16=8 / 4,
# where trace.coop_lanes 16 runs groups of 8 / 4 lanes) and step cap.
# usage (GPU box): bash tools/coop_g_sweep.sh "lib:lanes ..." "caps" [rounds]
set -o pipefail
libs=${1:-"librtamd.so:32 exp/cg8.so:16 exp/cg4.so:16"}
caps=${2:-"24 36 48 72"}
rounds=${3:-1}
for r in $(seq 1 $rounds); do
  for cap in $caps; do
    for spec in $libs; do
      lib=${spec%%:*}; lanes=${spec##*:}
      out=$(RT_LIB=$PWD/gpu_raytracer_amd/lib/$lib timeout -k 10 120 python tools/rank_emul.py config=3 frames=6 \
            ranks=8 trace.coop_cap_tiles=$cap trace.coop_lanes=$lanes 2>/dev/null) || { echo "FAILED $lib $cap"; exit 1; }
      echo "$out" | python -c "import json,sys; d=json.load(sys.stdin); p=d['P']['8']; print(f'round $r cap $cap $lib lanes $lanes: P=8 max {p[\"max_ms\"]:.4f} mean {p[\"mean_ms\"]:.4f} ms, full {d[\"full_frame_ms\"]:.4f}', flush=True)"
    done
  done
done
