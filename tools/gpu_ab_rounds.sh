#!/bin/bash
# GPU box: interleaved A/B of bench.py over the product library and experiment libraries
# lib/exp/NAME.so (PBRTGPU_LIB), ROUNDS rounds so box noise shows.
# Usage: bash tools/gpu_ab_rounds.sh TAG ROUNDS "bench args" NAME...
set -e
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for e in cur "$@"; do
    L=""; [ $e != cur ] && L=$PWD/pbrt-v2-spectral_amd/lib/exp/$e.so
    PBRTGPU_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu --no-slices $ARGS > $OUT/${e}_$r.json 2> $OUT/${e}_$r.err || { tail -5 $OUT/${e}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/${e}_$r.json')); print('$e', $r, d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
  done
done
