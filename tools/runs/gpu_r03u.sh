#!/bin/bash
# GPU suite with the whole-pool slot rule, then C2 (slices included), C1 and C2 DirectLighting
# under the new rule and the round-2 rule (PBRTGPU_SLOT_DIV=4)
set -e
OUT=$PWD/gpurun_out/r03u
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
b() {   # name, bench args
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { tail -20 $OUT/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$n.json')); r=d.get('roofline') or {}; print('$n', d['value'], d['ms_per_step'], r.get('frac'), r.get('traffic'), {k: v['efficiency'] for k, v in (d.get('slice_efficiency') or {}).items() if isinstance(v, dict)})"
}
b c2 --steps 5 --warmup 2
for dv in 1 4; do
  export PBRTGPU_SLOT_DIV=$dv
  b c1_div$dv --config c1 --steps 5 --warmup 2 --no-cpu --no-slices --no-roofline
  b c2_slices_div$dv --steps 3 --warmup 1 --no-cpu --no-roofline
  b c2_dl_div$dv --integrator directlighting --strategy all --steps 2 --no-cpu --no-slices --no-roofline
done
