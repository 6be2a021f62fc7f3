#!/bin/bash
# GPU-box: selected parity tests (-k expression) then bench on the given configs.
# Usage: bash tools/gpu_cfg.sh TAG "pytest -k expr" c2 [c3 ...]
set -e
TAG=$1; K=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --config $c --steps 1 --no-cpu > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$c.json')); r=d['roofline']
print('$c', d['value'], 'Mpaths/s', d['ms_per_step'], 'ms/step', 'serial', r['serial_frame_ms'], {k: v['ms_per_frame'] for k, v in r['kernels'].items()})"
done
