#!/bin/bash
# per-pass log of C2 slices; per-config rocprof profiles (trace + PMC), summarised on the box
set -e
mkdir -p gpurun_out/r03p
NS=8,1 PBRTGPU_PASS_LOG=1 timeout -k 10 200 python3 tools/slice_timing.py > gpurun_out/r03p/slices.log 2> gpurun_out/r03p/passes.log
bash tools/gpu_profile.sh r03p_c3 c3
bash tools/gpu_profile.sh r03p_c4 c4
bash tools/gpu_profile.sh r03p_c5 c5
bash tools/gpu_profile.sh r03p_dl c2 --integrator directlighting --strategy all
bash tools/gpu_profile.sh r03p_c2 c2
du -sh gpurun_out
