#!/bin/bash
# r05f: GPU suite (spot / distant lights, ABI 15, 60-band FEAT 0 DirectLighting kernels at 2
# waves/SIMD); the 60-band DirectLighting kernels at 2 vs 1 waves/SIMD (lib/exp/dl60w1.so: the same
# tree with the 1-wave k_dl_nee / k_dl_spec) on C2's scene in the 60-band build, twice each
OUT=$PWD/gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c2_b60 --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl60_w2_$r.json 2> $OUT/bench_dl60_w2_$r.err || { tail -20 $OUT/bench_dl60_w2_$r.err; exit 1; }
  cut -c1-200 $OUT/bench_dl60_w2_$r.json
  PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/dl60w1.so timeout -k 10 300 python3 bench.py --config c2_b60 --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl60_w1_$r.json 2> $OUT/bench_dl60_w1_$r.err || { tail -20 $OUT/bench_dl60_w1_$r.err; exit 1; }
  cut -c1-200 $OUT/bench_dl60_w1_$r.json
done
timeout -k 10 300 python3 bench.py --config c2_b60 --no-cpu --no-slices > $OUT/bench_c2_b60.json 2> $OUT/bench_c2_b60.err || { tail -20 $OUT/bench_c2_b60.err; exit 1; }
cut -c1-200 $OUT/bench_c2_b60.json
echo done
