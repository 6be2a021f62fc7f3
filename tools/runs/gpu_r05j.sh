#!/bin/bash
# r05j: the final tree as the driver runs it -- GPU suite, smoke, `python bench.py` (defaults:
# C2 with roofline, CPU baseline and slices) -- then C2 DirectLighting, the 60-band DirectLighting
# line (k_dl_nee at 2 waves, k_dl_spec at 1) and C3
OUT=$PWD/gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -5 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cut -c1-300 $OUT/bench_default.json
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl.json 2> $OUT/bench_dl.err || { tail -20 $OUT/bench_dl.err; exit 1; }
cut -c1-200 $OUT/bench_dl.json
timeout -k 10 300 python3 bench.py --config c2_b60 --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl60.json 2> $OUT/bench_dl60.err || { tail -20 $OUT/bench_dl60.err; exit 1; }
cut -c1-200 $OUT/bench_dl60.json
timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
cut -c1-200 $OUT/bench_c3.json
echo done
