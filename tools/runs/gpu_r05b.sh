#!/bin/bash
# r05b: GPU suite with every parity assertion at bit equality (plus the gpupath end-to-end
# test through the reference's own film); the XCD-contiguous trace ranges A/B (C2 and C2
# DirectLighting, two interleaved rounds, slices, TCC hit rates); the band-count experiment
# (k_shade at 16 bands on the 32-band scene: the cost of per-lane band work at equal occupancy)
OUT=$PWD/gpurun_out/r05b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -40 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for x in 0 1; do
    PBRTGPU_XCD_MAP=$x timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench_c2_xcd${x}_$r.json 2> $OUT/bench_c2_xcd${x}_$r.err || { tail -20 $OUT/bench_c2_xcd${x}_$r.err; exit 1; }
    cut -c1-200 $OUT/bench_c2_xcd${x}_$r.json
  done
done
for x in 0 1; do
  PBRTGPU_XCD_MAP=$x timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl_xcd$x.json 2> $OUT/bench_dl_xcd$x.err || { tail -20 $OUT/bench_dl_xcd$x.err; exit 1; }
  cut -c1-200 $OUT/bench_dl_xcd$x.json
  PBRTGPU_XCD_MAP=$x timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc_$x -o run -- python3 bench.py --no-cpu --no-roofline --no-slices --steps 1 --warmup 0 --serial > $OUT/pmc_tcc_$x.json 2> $OUT/pmc_tcc_$x.err || { tail -20 $OUT/pmc_tcc_$x.err; exit 1; }
  python3 tools/pmc_table.py $OUT/pmc_tcc_$x > $OUT/pmc_tcc_$x.txt 2>&1
  rm -rf $OUT/pmc_tcc_$x
done
for e in cur nbhalf3 nbhalf4; do
  PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/$e.so timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_exp_$e.json 2> $OUT/bench_exp_$e.err || { tail -20 $OUT/bench_exp_$e.err; exit 1; }
  cut -c1-200 $OUT/bench_exp_$e.json
done
echo done
