#!/bin/bash
# Per-kernel VGPRs / occupancy / scratch of one .hip file (compile-time remarks).
# usage: tools/kres.sh gpu_raytracer_amd/csrc/trace_kernels.hip [name filter]
F=$1; PAT=${2:-.}; EXTRA=${KRES_FLAGS:-}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 $EXTRA -c "$F" -o /tmp/kres.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 | awk '
/Function Name:/ {n=$NF; sub(/\[.*/,"",n); name=$0; sub(/.*Function Name: /,"",name); sub(/ \[-Rpass.*/,"",name)}
/ VGPRs:/ {v=$0; sub(/.*VGPRs: /,"",v); sub(/ \[.*/,"",v)}
/ScratchSize/ {s=$0; sub(/.*lane\]: /,"",s); sub(/ \[.*/,"",s)}
/Occupancy/ {o=$0; sub(/.*SIMD\]: /,"",o); sub(/ \[.*/,"",o); printf "%-4s vgpr %-4s occ %-3s scratch %s\n", "", v, o, s; print "     " substr(name,1,90)}' | paste - - | grep -E "$PAT"
