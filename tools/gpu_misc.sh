#!/bin/bash
# wide-record tests + build stage times + the tile-order A/B for per-rank tiles
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_wide8_gpu.py tests/test_parity_gpu.py tests/test_dbuild_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_misc.log 2>&1
rc=$?; tail -2 gpurun_out/t_misc.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_misc.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/build_times.py > gpurun_out/build_times.log 2>&1 || { tail -5 gpurun_out/build_times.log; exit 1; }
tail -6 gpurun_out/build_times.log
MODES=p2,p4,p8 bash tools/gpu_ab2.sh gpu_raytracer_amd/lib/librtamd.so gpu_raytracer_amd/lib/librtamd.so@trace.tile_order=0
timeout -k 10 300 python -u tools/order_bound.py 16 3 2>&1 | grep -v amdgpu.ids
