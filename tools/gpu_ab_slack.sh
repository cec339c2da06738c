#!/bin/bash
# GPU pass: parity of the per-ray record slack (wide, 8-ary, coop, shadow, path,
# headline), then the library A/B (HEAD~ baseline vs per-ray slack vs forced 6 waves).
mkdir -p gpurun_out
export TMPDIR=/tmp
true
rc=0
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error|assert" gpurun_out/t_slack.log | head -20; exit $rc; }
L=gpu_raytracer_amd/lib
timeout -k 10 600 python -u tools/ab_libs.py 3 moving,trace,p8,shadow,path,build $L/exp/base.so $L/librtamd.so $L/exp/slack_w6.so "$L/librtamd.so@build.wide_arity=8" > gpurun_out/ab_slack.log 2>&1 || { tail -20 gpurun_out/ab_slack.log; exit 1; }
tail -8 gpurun_out/ab_slack.log
