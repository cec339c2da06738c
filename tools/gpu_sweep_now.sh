#!/bin/bash
# coop cap / lane sweeps on the current tree (per-rank tiles, soup-1M 1080p)
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in ${LANES:-16 64}; do
timeout -k 10 300 python -u tools/coop_sweep.py 1000000 1920 1080 1 ${ROUNDS:-3} ${CAPS:-0 1 8 16 32 48 64 80 96} trace.coop_lanes=$L > gpurun_out/sweep_l$L.log 2>&1 || { tail -20 gpurun_out/sweep_l$L.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sweep_l$L.log
done
