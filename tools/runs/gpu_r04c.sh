#!/bin/bash
# r04c: C2 A/B of the A / B band loops (experiment lib with the loops skipped: the upper bound of
# a scalar A / B form), then the C2 profile of the 4-wide build (kernel trace, PMC incl. TCC hit
# rate) and the TCC pass with the 4-wide queries off
OUT=$PWD/gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/noabloop.so timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_noabloop.json 2> $OUT/bench_c2_noabloop.err || { tail -20 $OUT/bench_c2_noabloop.err; exit 1; }
cat $OUT/bench_c2_noabloop.json
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_again.json 2> $OUT/bench_c2_again.err || exit 1
cat $OUT/bench_c2_again.json
bash tools/gpu_profile.sh r04c_c2 c2 > $OUT/profile.log 2>&1 || { tail -20 $OUT/profile.log; exit 1; }
B="bench.py --config c2 --no-cpu --no-roofline --no-slices"
PBRTGPU_SHADOW4=0 PBRTGPU_CLOSEST4=0 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/w4off_tcc -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/w4off_tcc.json 2> $OUT/w4off_tcc.err || echo "TCC pass (w4 off) failed"
ls gpurun_out/summaries
