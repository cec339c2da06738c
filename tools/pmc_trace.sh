#!/bin/bash
# PMC passes on the trace kernel (tools/trace_only.py); one counter group per
# pass.  Usage: bash tools/pmc_trace.sh <tag> [trace.variant]
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-trace}
VAR=${2:-0}
mkdir -p $OUT
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
  "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE" \
  "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ" \
  "TCC_HIT TCC_MISS" \
  "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS"; do
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -- python3 tools/trace_only.py 3 $VAR > $OUT/p$i.log 2>&1
  i=$((i+1))
done
echo pmc done
