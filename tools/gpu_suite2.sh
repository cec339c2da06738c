#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/suite_$r.log 2>&1; echo "suite $r rc=$?"; tail -1 gpurun_out/suite_$r.log; grep -E "prims differ|^FAILED" gpurun_out/suite_$r.log | head -5
done
timeout -k 10 500 python -u tools/stress_render.py 400 7 > gpurun_out/stress2.log 2>&1; tail -1 gpurun_out/stress2.log
