#!/bin/bash
# rocprof kernel traces + PMC passes of every config with the final round-3 build (16 M slot target)
set -e
mkdir -p gpurun_out
bash tools/gpu_profile.sh r03ag_c2 c2
bash tools/gpu_profile.sh r03ag_dl c2 --integrator directlighting --strategy all
bash tools/gpu_profile.sh r03ag_c5 c5
bash tools/gpu_profile.sh r03ag_c4 c4
bash tools/gpu_profile.sh r03ag_c3 c3
du -sh gpurun_out
