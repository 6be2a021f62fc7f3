#!/bin/bash
# r06ai: the straight-line trace kernels at 6 waves/SIMD -- lib/exp/s6 (k_trace_s4: 80 VGPRs, 6
# spilled) and lib/exp/cs6 (k_trace_s4 and k_trace_c4: 80 VGPRs, 6 / 19 spilled) against the product
# library (5 waves: 88 / 93 VGPRs) on C2 and C2 DirectLighting
OUT=$PWD/gpurun_out/r06ai
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06ai/ab_c2 2 "--config c2" s6 cs6 || exit 1
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06ai/ab_dl 2 "--config c2 --integrator directlighting" s6 cs6 || exit 1
echo done
