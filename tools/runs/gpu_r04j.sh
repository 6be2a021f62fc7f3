#!/bin/bash
# r04j: normal maps, animated camera (pack v13) -- GPU suite incl.
# the imagemap goldens, then the C2 / C4 bench lines
OUT=$PWD/gpurun_out/r04j
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-slices > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
