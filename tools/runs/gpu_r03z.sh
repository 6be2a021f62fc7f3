#!/bin/bash
# GPU suite (with the render-setup cache test), then C2 twice with slices (adaptive pass batch)
set -e
OUT=$PWD/gpurun_out/r03z
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_c2_$r.json 2> $OUT/bench_c2_$r.err || { tail -20 $OUT/bench_c2_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c2_$r.json')); r=d['roofline']; print('c2', $r, d['value'], d['ms_per_step'], r['frac'], r['traffic'], {k: (v['efficiency'], v['passes']) for k, v in d['slice_efficiency'].items() if isinstance(v, dict)})"
done
