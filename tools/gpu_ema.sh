#!/bin/bash
# running-mean tile order: the trace/coop/multi-GPU GPU tests on the in-tree library
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_coop_gpu.py tests/test_multi_gpu.py tests/test_wide8_gpu.py tests/test_shadow_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ema.log 2>&1 || { tail -30 gpurun_out/t_ema.log; exit 1; }
tail -1 gpurun_out/t_ema.log
