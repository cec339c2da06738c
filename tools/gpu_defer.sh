#!/bin/bash
# GPU pass: leaf-deferral parity, then the A/B of trace.leaf_defer thresholds.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_coop_gpu.py tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_defer.log 2>&1
rc=$?; tail -3 gpurun_out/t_defer.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_defer.log | head -20; exit $rc; }
L=gpu_raytracer_amd/lib/librtamd.so
timeout -k 10 600 python -u tools/ab_libs.py 3 moving,trace,p8 $L "$L@trace.leaf_defer=16" "$L@trace.leaf_defer=24" "$L@trace.leaf_defer=32" "$L@trace.leaf_defer=48" > gpurun_out/ab_defer.log 2>&1 || { tail -20 gpurun_out/ab_defer.log; exit 1; }
tail -7 gpurun_out/ab_defer.log
