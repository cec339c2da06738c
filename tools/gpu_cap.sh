#!/bin/bash
# coop + multi-GPU tests, then per-rank spread with the default (auto) cap
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_coop_gpu.py tests/test_multi_gpu.py tests/test_wide8_gpu.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_cap.log 2>&1 || { tail -30 gpurun_out/t_cap.log; exit 1; }
tail -2 gpurun_out/t_cap.log
timeout -k 10 120 python -u tools/rank_spread.py > gpurun_out/spread_auto.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/spread_auto.log
