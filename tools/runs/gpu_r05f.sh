#!/bin/bash
# r05f: GPU suite (spot / distant lights, the orthographic camera, ABI 15, 60-band FEAT 0
# DirectLighting kernels at 2 waves/SIMD); the 60-band DirectLighting kernels at 2 vs 1 waves/SIMD
# (lib/exp/dl60w1.so: the same tree with 1-wave k_dl_nee / k_dl_spec) on C2's scene in the 60-band
# build; C2 with three wavefront lanes (lib/exp/lanes3.so) and with 8 hardware queues per process
OUT=$PWD/gpurun_out/r05f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
X=$PWD/pbrt-v2-spectral_amd/lib/exp
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c2_b60 --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl60_w2_$r.json 2> $OUT/bench_dl60_w2_$r.err || { tail -20 $OUT/bench_dl60_w2_$r.err; exit 1; }
  cut -c1-200 $OUT/bench_dl60_w2_$r.json
  PBRTGPU_LIB=$X/dl60w1.so timeout -k 10 300 python3 bench.py --config c2_b60 --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl60_w1_$r.json 2> $OUT/bench_dl60_w1_$r.err || { tail -20 $OUT/bench_dl60_w1_$r.err; exit 1; }
  cut -c1-200 $OUT/bench_dl60_w1_$r.json
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_l2_q${q}_$r.json 2> $OUT/bench_c2_l2_q${q}_$r.err || { tail -20 $OUT/bench_c2_l2_q${q}_$r.err; exit 1; }
    cut -c1-200 $OUT/bench_c2_l2_q${q}_$r.json
    GPU_MAX_HW_QUEUES=$q PBRTGPU_LIB=$X/lanes3.so timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_l3_q${q}_$r.json 2> $OUT/bench_c2_l3_q${q}_$r.err || { tail -20 $OUT/bench_c2_l3_q${q}_$r.err; exit 1; }
    cut -c1-200 $OUT/bench_c2_l3_q${q}_$r.json
  done
done
timeout -k 10 300 python3 bench.py --config c2_b60 --no-cpu --no-slices > $OUT/bench_c2_b60.json 2> $OUT/bench_c2_b60.err || { tail -20 $OUT/bench_c2_b60.err; exit 1; }
cut -c1-200 $OUT/bench_c2_b60.json
echo done
