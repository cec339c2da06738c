#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_coop_gpu.py tests/test_parity_gpu.py tests/test_multi_gpu.py tests/test_wide8_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ord.log 2>&1
rc=$?; tail -2 gpurun_out/t_ord.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_ord.log | head -20; exit $rc; }
MODES=p2,p4,p8 bash tools/gpu_ab2.sh gpu_raytracer_amd/lib/exp/head.so gpu_raytracer_amd/lib/librtamd.so
