#!/bin/bash
# A/B of two library builds (args: lib paths relative to the repo) on the headline modes
mkdir -p gpurun_out
export TMPDIR=/tmp
MODES=${MODES:-moving,trace,p8,build}
timeout -k 10 600 python -u tools/ab_libs.py 4 $MODES "$@" > gpurun_out/ab2.log 2>&1 || { tail -20 gpurun_out/ab2.log; exit 1; }
tail -5 gpurun_out/ab2.log
