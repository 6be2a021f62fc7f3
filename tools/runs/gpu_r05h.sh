#!/bin/bash
# r05h: GPU suite (heightfield shapes, metadata mesh ids over them); k_trace_s4 alone at 6
# waves/SIMD (lib/exp/s6.so) against the product, C2 and C2 DirectLighting, two interleaved rounds
OUT=$PWD/gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
X=$PWD/pbrt-v2-spectral_amd/lib/exp
for r in 1 2; do
  for v in base s6; do
    L=""; [ $v != base ] && L="PBRTGPU_LIB=$X/$v.so"
    env $L timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_${v}_$r.json 2> $OUT/bench_c2_${v}_$r.err || { tail -20 $OUT/bench_c2_${v}_$r.err; exit 1; }
    cut -c1-160 $OUT/bench_c2_${v}_$r.json
    env $L timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl_${v}_$r.json 2> $OUT/bench_dl_${v}_$r.err || { tail -20 $OUT/bench_dl_${v}_$r.err; exit 1; }
    cut -c1-160 $OUT/bench_dl_${v}_$r.json
  done
done
echo done
