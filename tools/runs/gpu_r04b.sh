#!/bin/bash
# r04b: glibc-exact transcendentals, the full-spp window parity tests, the light-field / eye
# cameras, the 4-wide BVH copy (k_trace_s4 / k_trace_c4) -- GPU suite, then C2 bench lines with the
# 4-wide queries on, off, shadow only (A/B on one box), then a rocprof kernel-trace of the C2 bench
OUT=$PWD/gpurun_out/r04b
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
PBRTGPU_SHADOW4=0 PBRTGPU_CLOSEST4=0 timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_w4off.json 2> $OUT/bench_c2_w4off.err || { tail -20 $OUT/bench_c2_w4off.err; exit 1; }
cat $OUT/bench_c2_w4off.json
PBRTGPU_CLOSEST4=0 timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_c4off.json 2> $OUT/bench_c2_c4off.err || { tail -20 $OUT/bench_c2_c4off.err; exit 1; }
cat $OUT/bench_c2_c4off.json
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_again.json 2> $OUT/bench_c2_again.err || exit 1
cat $OUT/bench_c2_again.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-slices --no-roofline --serial > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
ls -R $OUT/prof | head -20
