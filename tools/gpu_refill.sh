#!/bin/bash
# parity tests, then bench at several ray-replacement thresholds.  Usage: bash tools/gpu_refill.sh TAG
set -e
OUT=$PWD/gpurun_out/${1:-refill}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in ${REFILLS:-4 8 16 32 64}; do
  PBRTGPU_REFILL=$r timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/r$r.json
  python3 -c "import json; d=json.load(open('$OUT/r$r.json')); print('refill $r', d['value'], d['roofline']['kernel_ms_per_step'])"
done
