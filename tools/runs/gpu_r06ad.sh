#!/bin/bash
# r06ad: the FEAT_BASIC k_shade forced to 4 waves/SIMD (lib/exp/w4: 128 VGPRs, 143 spilled) against
# the product library (3 waves, 168 VGPRs, 9 spilled) on C2, two rounds
OUT=$PWD/gpurun_out/r06ad
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06ad/ab_c2 2 "--config c2" w4 || exit 1
echo done
