"""Per-kernel VGPR / LDS / occupancy of a .hip file (compiler remarks).
    python tools/kres.py gpu_raytracer_amd/csrc/trace_kernels.hip [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-fno-fast-math",
                      "-fPIC", "-std=c++17", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|VGPRs Spill): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split(" [")[0]] = int(m.group(2))
dem = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.splitlines()
for (k, v), d in zip(rows.items(), dem):
    if flt in d:
        d = re.sub(r"\(.*", "", d)
        print(f"{d:70s} VGPR {v.get('VGPRs')} spill {v.get('VGPRs Spill')} LDS {v.get('LDS Size')} occ {v.get('Occupancy')} scratch {v.get('ScratchSize')}")
