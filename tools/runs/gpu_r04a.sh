#!/bin/bash
# r04a: glibc-exact transcendentals (include/pbrt_libmf.h) -- GPU suite incl. the full-spp window
# parity tests and the libm hook, then the default bench line
OUT=$PWD/gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -40 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
T0=$(date +%s); timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "bench wall: $(( $(date +%s) - T0 )) s"
