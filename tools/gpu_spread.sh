#!/bin/bash
# rank spread + low-cap coop sweep (lanes 16 and 32) on the current library
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/rank_spread.py > gpurun_out/spread.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/coop_sweep.py 1000000 1920 1080 1 3 0 48 56 64 72 80 trace.coop_lanes=32 > gpurun_out/sweep_low32.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/coop_sweep.py 1000000 1920 1080 1 3 0 48 56 64 72 80 trace.coop_lanes=16 > gpurun_out/sweep_low16.log 2>&1 || exit 1
