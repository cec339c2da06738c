#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in head.so cur; do
  for r in 1 2; do
    if [ $L = cur ]; then unset RT_LIB; else export RT_LIB=$PWD/gpu_raytracer_amd/lib/exp/$L; fi
    timeout -k 10 200 python -u -m pytest tests/test_wide8_gpu.py -m gpu -q --timeout 120 --timeout-method thread -k "presets_and_zero" > gpurun_out/w8_${L}_$r.log 2>&1; echo "$L run $r rc=$?"; tail -1 gpurun_out/w8_${L}_$r.log
  done
done
unset RT_LIB
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_coop_gpu.py tests/test_multi_gpu.py tests/test_wide8_gpu.py -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/w8_seq.log 2>&1; echo "seq rc=$?"; tail -1 gpurun_out/w8_seq.log
