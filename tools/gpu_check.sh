#!/bin/bash
# One GPU-box pass: gpu tests, the headline bench, the spawned 2-rank gloo
# rehearsal.  Usage: bash tools/gpu_check.sh <tag> [pytest -k expr]
TAG=${1:-r02}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KA[@]}" > gpurun_out/t_$TAG.log 2>&1
rc=$?
tail -3 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error|error" gpurun_out/t_$TAG.log | head -20; exit $rc; }
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-600 gpurun_out/bench_$TAG.json
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --steps 5 --no-cpu-baseline --no-extra > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err || { tail -20 gpurun_out/bench2_$TAG.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench2_$TAG.json').read().strip().splitlines()[-1]);print('N=2 gloo', d['value'], d['image_crc32'])"
