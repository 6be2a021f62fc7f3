#!/bin/bash
# GPU suite, C2 bench (slices), C1, then one GPU's 1/2, 1/4, 1/8 of C2 and the whole frame (min of 3) with the final slot rule
set -e
OUT=$PWD/gpurun_out/r03af
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu > $OUT/bench_c2_$r.json 2> $OUT/bench_c2_$r.err || { tail -20 $OUT/bench_c2_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_c2_$r.json')); r=d['roofline']; print('c2', $r, d['value'], d['ms_per_step'], r['frac'], {k: (v['efficiency'], v['passes'], v['Mpaths_s']) for k, v in d['slice_efficiency'].items() if isinstance(v, dict)})"
done
timeout -k 10 300 python3 bench.py --config c1 --steps 5 --warmup 2 --no-cpu --no-slices --no-roofline > $OUT/bench_c1.json 2> $OUT/bench_c1.err || { tail -20 $OUT/bench_c1.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_c1.json')); print('c1', d['value'], d['ms_per_step'])"
NS=2,4,8,1 timeout -k 10 200 python3 tools/slice_timing.py > $OUT/slices.log 2>&1 || { tail -5 $OUT/slices.log; exit 1; }
grep frame $OUT/slices.log
