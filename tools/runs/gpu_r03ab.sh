#!/bin/bash
# rocprof kernel traces + PMC passes of C3, C4, C5 with the final round-3 build
set -e
mkdir -p gpurun_out
bash tools/gpu_profile.sh r03ab_c5 c5
bash tools/gpu_profile.sh r03ab_c4 c4
bash tools/gpu_profile.sh r03ab_c3 c3
du -sh gpurun_out
