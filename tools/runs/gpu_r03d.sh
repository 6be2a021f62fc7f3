#!/bin/bash
set -e
OUT=$PWD/gpurun_out/r03d
mkdir -p $OUT
bash tools/gpu_ab_trace.sh r03d/dl "--integrator directlighting --strategy all" prev
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/sections.so timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-roofline --serial > $OUT/sections.json 2> $OUT/sections.err
grep sections $OUT/sections.err
