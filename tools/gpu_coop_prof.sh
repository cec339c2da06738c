#!/bin/bash
mkdir -p gpurun_out/coop_prof
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/coop_prof -- python3 tools/coop_prof.py "$@" > gpurun_out/coop_prof.log 2>&1 || { tail gpurun_out/coop_prof.log; exit 1; }
python3 tools/coop_prof_parse.py gpurun_out/coop_prof "$@"
