#!/bin/bash
# GPU box: k_shade section timing (experiment libraries lib/exp/sec*.so built with -DPGD_SECTIONS)
# over one serial frame.  Usage: bash tools/gpu_sections.sh TAG [bench args...]
set -e
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for v in pbrt-v2-spectral_amd/lib/exp/sec*.so; do
  n=$(basename $v .so)
  PBRTGPU_LIB=$PWD/$v timeout -k 10 200 python3 bench.py --steps 1 --warmup 0 --no-cpu --no-roofline --serial "$@" > $OUT/$n.json 2> $OUT/$n.err
  echo "$n: $(grep sections $OUT/$n.err)"
done
