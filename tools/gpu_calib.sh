#!/bin/bash
# FETCH_SIZE calibration for the random 36-B gather (tools/calib_gather.hip)
mkdir -p gpurun_out/calib
export TMPDIR=/tmp
B=tools/build/calib_gather
timeout -k 10 60 ./$B 1000000 3 > gpurun_out/calib/run.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -- ./$B 1000000 3 > gpurun_out/calib/fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/calib/req -- ./$B 1000000 3 > gpurun_out/calib/req.log 2>&1 || echo "req pass failed"
timeout -k 10 120 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/calib/hit -- ./$B 1000000 3 > gpurun_out/calib/hit.log 2>&1 || echo "hit pass failed"
echo calib done
