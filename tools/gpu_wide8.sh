#!/bin/bash
# GPU pass for the 8-ary records: their parity tests and the wide tests, then
# the arity A/B and the coop cap sweep at arity 8.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_wide8_gpu.py tests/test_wide_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_wide8.log 2>&1
rc=$?; tail -3 gpurun_out/t_wide8.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_wide8.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/ab_arity.py 3 12 > gpurun_out/ab_arity.log 2>&1 || { tail -20 gpurun_out/ab_arity.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ab_arity.log
timeout -k 10 300 python -u tools/coop_sweep.py 1000000 1920 1080 1 3 0 32 48 64 96 build.wide_arity=8 > gpurun_out/coop_sweep8.log 2>&1 || { tail -20 gpurun_out/coop_sweep8.log; exit 1; }
grep -v amdgpu.ids gpurun_out/coop_sweep8.log
