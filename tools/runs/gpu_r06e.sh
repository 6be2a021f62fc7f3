#!/bin/bash
# r06e: k_shade section timing (lib/exp/sec*.so, -DPGD_SECTIONS [-DPGD_SECTIONS_DRAIN]) of one serial
# C2 frame and one serial C3 frame in the current tree
OUT=$PWD/gpurun_out/r06e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 bash tools/gpu_sections.sh r06e/c2 --config c2 || exit 1
timeout -k 10 400 bash tools/gpu_sections.sh r06e/c3 --config c3 || exit 1
echo done
