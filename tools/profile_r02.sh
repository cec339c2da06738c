#!/bin/bash
# On the GPU box (via gpurun): kernel trace + three PMC passes of the timed
# bench steps (bench.py --only-timed) for one config; FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950 and the SQ group takes a third.
# Usage: bash tools/profile_r02.sh <tag> <config key> <steps>
# Then, here: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag> <config name> 3
TAG=$1; CFG=${2:-3}; STEPS=${3:-20}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="bench.py --only-timed --no-cpu-baseline --no-extra --config $CFG --steps $STEPS --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -- python3 $B > $OUT/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -- python3 $B > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -- python3 $B > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -- python3 $B > $OUT/sq.log 2>&1 || exit 1
echo "profile $TAG done"
