#!/bin/bash
# GPU box: bench.py with the product library and every experiment library in lib/exp (PBRTGPU_LIB).
# Usage: bash tools/gpu_exp_bench.sh TAG [bench args...]
set -e
TAG=$1; shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
shopt -s nullglob
for v in cur pbrt-v2-spectral_amd/lib/exp/*.so; do
  n=$(basename $v .so); L=""; [ $v != cur ] && L=$PWD/$v
  PBRTGPU_LIB=$L timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu --no-slices "$@" > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
done
