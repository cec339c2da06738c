#!/bin/bash
# reprojected tile/pixel order: its parity tests, the order bound, the moving A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_coop_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_rp.log 2>&1
rc=$?; tail -2 gpurun_out/t_rp.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_rp.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/order_bound.py 16 3 2>&1 | grep -v amdgpu.ids
