#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_coop_gpu.py tests/test_multi_gpu.py tests/test_wide8_gpu.py tests/test_shadow_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/w8rep_$r.log 2>&1; echo "run $r rc=$?"; tail -1 gpurun_out/w8rep_$r.log; grep -E "prims differ|^FAILED" gpurun_out/w8rep_$r.log | head -5
done
