#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/stress_render.py 1500 11 > gpurun_out/stress_final.log 2>&1; tail -1 gpurun_out/stress_final.log; grep -c MISMATCH gpurun_out/stress_final.log
for r in 1 2 3 4 5; do
  timeout -k 10 200 python -u -m pytest tests/test_wide8_gpu.py tests/test_wide_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/w8final_$r.log 2>&1; echo "wide run $r rc=$?"; tail -1 gpurun_out/w8final_$r.log
done
