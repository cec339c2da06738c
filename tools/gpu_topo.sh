#!/bin/bash
# build parity tests + build-time A/B (head vs working tree)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_wide_gpu.py tests/test_wide8_gpu.py tests/test_dbuild_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_topo.log 2>&1 || { tail -30 gpurun_out/t_topo.log; exit 1; }
tail -2 gpurun_out/t_topo.log
bash tools/gpu_buildab.sh gpu_raytracer_amd/lib/exp/head.so gpu_raytracer_amd/lib/exp/topo.so > gpurun_out/buildab_topo.log 2>&1
