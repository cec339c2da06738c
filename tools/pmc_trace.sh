#!/bin/bash
# PMC passes on the trace kernel (tools/trace_only.py); one counter group per pass.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${1:-trace}
mkdir -p $OUT
i=${2:-1}
for grp in \
  "TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS GRBM_GUI_ACTIVE" \
  "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES" \
  "TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ" \
  "TCC_HIT TCC_MISS" \
  "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH"; do
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -- python3 tools/trace_only.py 3 > $OUT/p$i.log 2>&1
  i=$((i+1))
done
echo pmc done
