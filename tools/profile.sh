#!/bin/bash
# Run on the GPU box (via gpurun): kernel-trace stats + two PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950).
# Usage: bash tools/profile.sh <tag> [bench args...]
set -e
TAG=${1:-r01}; shift || true
ARGS=${@:-"--steps 20 --warmup 3 --no-cpu-baseline"}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python3 bench.py $ARGS > $OUT/bench_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -- python3 bench.py $ARGS > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -- python3 bench.py $ARGS > $OUT/bench_write.log 2>&1
echo profile done
