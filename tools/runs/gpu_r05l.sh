#!/bin/bash
# r05l: C3 with the compact kd nodes walked with branches (PBRTGPU_KD_COMPACT=2) against the
# select-based walk (1) and the two-float4 nodes (0), interleaved
OUT=$PWD/gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -rf -k "measured" > $OUT/pytest_kd.log 2>&1
rc=$?
tail -5 $OUT/pytest_kd.log
[ $rc -le 1 ] || exit $rc
for m in 2 0 1 2 0; do
PBRTGPU_KD_COMPACT=$m timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3_m$m.json 2> $OUT/bench_c3_m$m.err || { tail -20 $OUT/bench_c3_m$m.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c3_m$m.json'));k=d['roofline']['kernels'];print('m$m',d['value'],k['k_shade']['ms_per_frame'])"
done
echo done
