#!/bin/bash
# GPU suite, then C2 (slices), C4, C1, C2 DirectLighting with the 16 M slot target and the half-of-items rule
set -e
OUT=$PWD/gpurun_out/r03ad
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { tail -20 $OUT/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$n.json')); r=d.get('roofline') or {}; print('$n', d['value'], d['ms_per_step'], r.get('frac'), {k: (v['efficiency'], v['passes'], v['Mpaths_s']) for k, v in (d.get('slice_efficiency') or {}).items() if isinstance(v, dict)})"
}
b c2 --steps 5 --warmup 2
b c2b --steps 5 --warmup 2 --no-cpu --no-roofline
b c4 --config c4 --steps 1 --no-cpu --no-slices
b c1 --config c1 --steps 5 --warmup 2 --no-cpu --no-slices
b c2_dl --integrator directlighting --strategy all --steps 2 --no-cpu --no-slices
b c5 --config c5 --steps 2 --no-cpu --no-slices
