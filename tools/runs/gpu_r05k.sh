#!/bin/bash
# r05k: the measured-BRDF walk over one-float4 kd nodes with the loop-free radius -- the C3 / kd
# parity tests, then C3 with the compact nodes (default) and with the two-float4 nodes
OUT=$PWD/gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_window_golden.py -m gpu -q --timeout 300 --timeout-method thread -rf -k "measured or bunny or c3 or meas or golden_keys" > $OUT/pytest_kd.log 2>&1
rc=$?
tail -15 $OUT/pytest_kd.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -20 $OUT/bench_c3.err; exit 1; }
cut -c1-200 $OUT/bench_c3.json
PBRTGPU_KD_COMPACT=0 timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3_wide.json 2> $OUT/bench_c3_wide.err || { tail -20 $OUT/bench_c3_wide.err; exit 1; }
cut -c1-200 $OUT/bench_c3_wide.json
timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3_b.json 2> $OUT/bench_c3_b.err || { tail -20 $OUT/bench_c3_b.err; exit 1; }
cut -c1-200 $OUT/bench_c3_b.json
echo done
