#!/bin/bash
# r05g: occupancy of the persistent trace kernels -- the product (k_trace_c4 94 / k_trace_s4 88
# VGPRs: 5 waves/SIMD) against builds forced to 6 (80 VGPRs) and 8 waves/SIMD (64 VGPRs, some
# scratch): C2 and C2 DirectLighting (1 G shadow rays per frame), two interleaved rounds
OUT=$PWD/gpurun_out/r05g
mkdir -p $OUT
export TMPDIR=/tmp
X=$PWD/pbrt-v2-spectral_amd/lib/exp
for r in 1 2; do
  for v in base tw6 tw8; do
    L=""; [ $v != base ] && L="PBRTGPU_LIB=$X/$v.so"
    env $L timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_${v}_$r.json 2> $OUT/bench_c2_${v}_$r.err || { tail -20 $OUT/bench_c2_${v}_$r.err; exit 1; }
    cut -c1-160 $OUT/bench_c2_${v}_$r.json
    env $L timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl_${v}_$r.json 2> $OUT/bench_dl_${v}_$r.err || { tail -20 $OUT/bench_dl_${v}_$r.err; exit 1; }
    cut -c1-160 $OUT/bench_dl_${v}_$r.json
  done
done
echo done
