#!/bin/bash
# GPU pass for the cooperative heavy-ray queue: its parity tests, then the cap sweep.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_coop_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_coop.log 2>&1
rc=$?; tail -3 gpurun_out/t_coop.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_coop.log | head -20; exit $rc; }
timeout -k 10 400 python -u tools/coop_sweep.py 1000000 1920 1080 1 3 > gpurun_out/coop_sweep.log 2>&1 || { tail -20 gpurun_out/coop_sweep.log; exit 1; }
cat gpurun_out/coop_sweep.log | grep -v amdgpu.ids
