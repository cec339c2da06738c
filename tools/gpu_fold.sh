#!/bin/bash
# the whole GPU suite on the in-tree library
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_fold.log 2>&1 || { tail -30 gpurun_out/t_fold.log; exit 1; }
tail -1 gpurun_out/t_fold.log
timeout -k 10 300 python -u tools/stress_render.py 300 3 > gpurun_out/stress3.log 2>&1; tail -1 gpurun_out/stress3.log
