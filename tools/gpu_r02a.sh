#!/bin/bash
# r02 GPU pass: tests, bench (N=1), N=2 gloo rehearsal, profiles of configs 3 and 5
bash tools/gpu_check.sh r02b || exit 1
bash tools/profile_r02.sh r02b_c3 3 20 || exit 1
bash tools/profile_r02.sh r02b_c5 5 6 || exit 1
