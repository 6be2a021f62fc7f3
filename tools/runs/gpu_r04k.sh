#!/bin/bash
# r04k: the DirectLighting light-sample list (k_dl_nee over the marked slots, batch rows) on top of r04j (normal maps, animated camera) -- GPU suite incl.
# the imagemap / animcam goldens, then bench lines of C2, C4, C3, C5 and C2 / C3 DirectLighting
OUT=$PWD/gpurun_out/r04k
mkdir -p $OUT
timeout -k 10 700 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-slices > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
timeout -k 10 300 python3 bench.py --config c5 --no-cpu --no-slices > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_c2_dl.json 2> $OUT/bench_c2_dl.err || { tail -20 $OUT/bench_c2_dl.err; exit 1; }
cat $OUT/bench_c2_dl.json
timeout -k 10 300 python3 bench.py --config c3 --integrator directlighting --no-cpu --no-slices > $OUT/bench_c3_dl.json 2> $OUT/bench_c3_dl.err || { tail -20 $OUT/bench_c3_dl.err; exit 1; }
cat $OUT/bench_c3_dl.json
