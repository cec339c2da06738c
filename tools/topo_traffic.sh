#!/bin/bash
# k_topo_refit's HBM traffic by stream, on the GPU box:
# FETCH_SIZE / WRITE_SIZE / TCC read-request passes of tools/build_times.py
# at n = 1M and 10M, for the shipped library and lib/exp/gseq.so (built by
# tools/build_exp.sh gseq "-DRT_EXP_GATHER_SEQ": leaf k's triangle read
# coalesced from tris[k], wrong output, traffic attribution only).
# -> gpurun_out/tt_<lib>_<n>_<pass>/ ; summarise with tools/topo_traffic.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 1000000 10000000; do
  for lib in librtamd.so exp/gseq.so; do
    tag=$(basename $lib .so)_$n
    for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
      p=$(echo $pass | cut -d' ' -f1)
      out=gpurun_out/tt_${tag}_$p
      timeout -k 10 -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $out -- \
        python3 tools/build_times.py $n 8 lib=gpu_raytracer_amd/lib/$lib > $out.log 2>&1 \
        || { echo "FAILED $tag $p"; tail -5 $out.log; exit 1; }
      echo "done $tag $p"
    done
  done
done
