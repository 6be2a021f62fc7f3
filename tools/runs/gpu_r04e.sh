#!/bin/bash
# r04e: C2 A/B on one box -- spectral A / B terms (lib/exp/spectral), deferred records (product),
# the A / B stores suppressed (lib/exp/noab), the A / B band loops skipped (lib/exp/noabloop)
OUT=$PWD/gpurun_out/r04e
mkdir -p $OUT
L=$PWD/pbrt-v2-spectral_amd/lib/exp
run() {   # name [lib]
  if [ -n "$2" ]; then export PBRTGPU_LIB=$2; else unset PBRTGPU_LIB; fi
  timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { tail -20 $OUT/bench_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$1.json')); k=d['roofline']['kernels']; print('$1', d['value'], {n: v['ms_per_frame'] for n, v in k.items()})"
}
run spectral $L/spectral.so && run deferred && run noab $L/noab.so && run noabloop $L/noabloop.so && run spectral2 $L/spectral.so && run deferred2
