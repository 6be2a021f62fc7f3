#!/bin/bash
# r05e: GPU suite (RGB build features, animated lens camera, quantized shadow walk goldens, C4
# whole frame); C3 with the one-walk kd-tree lookup (r05d: 343.8 Mpaths/s with two walks), twice;
# C2 and C2 DirectLighting lines of the same tree
OUT=$PWD/gpurun_out/r05e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3_$r.json 2> $OUT/bench_c3_$r.err || { tail -20 $OUT/bench_c3_$r.err; exit 1; }
  cut -c1-200 $OUT/bench_c3_$r.json
done
timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cut -c1-200 $OUT/bench_c2.json
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl.json 2> $OUT/bench_dl.err || { tail -20 $OUT/bench_dl.err; exit 1; }
cut -c1-200 $OUT/bench_dl.json
echo done
