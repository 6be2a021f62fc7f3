#!/bin/bash
# r04d: deferred A / B term records (wavefront.h DeferAB) -- GPU suite, then C2 bench lines
OUT=$PWD/gpurun_out/r04d
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_again.json 2> $OUT/bench_c2_again.err || exit 1
cat $OUT/bench_c2_again.json
timeout -k 10 300 python3 bench.py --config c5 --no-cpu --no-slices > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1
cat $OUT/bench_c5.json
