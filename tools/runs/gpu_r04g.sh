#!/bin/bash
# r04g: C2 A/B -- baseline (lib/exp/spectral), the exact shared-divisor division with its rerun
# (lib/exp/divexact), the fast form without fallback (lib/exp/divfast, timing only)
OUT=$PWD/gpurun_out/r04g
mkdir -p $OUT
L=$PWD/pbrt-v2-spectral_amd/lib/exp
run() {   # name lib
  export PBRTGPU_LIB=$2
  timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_$1.json 2> $OUT/bench_$1.err || { tail -20 $OUT/bench_$1.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$1.json')); k=d['roofline']['kernels']; print('$1', d['value'], {n: v['ms_per_frame'] for n, v in k.items()})"
}
run base $L/spectral.so && run divexact $L/divexact.so && run divfast $L/divfast.so && run base2 $L/spectral.so && run divexact2 $L/divexact.so
