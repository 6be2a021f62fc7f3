#!/bin/bash
# Round-3 record on one GPU box: GPU suite, smoke, bench lines of every config / integrator /
# renderer, then the C2 rocprof profile (kernel traces + PMC passes, summarised on the box)
set -e
OUT=$PWD/gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 120 python3 tools/gather_timing.py > $OUT/gather_timing.log 2>&1 || { tail -5 $OUT/gather_timing.log; exit 1; }
cat $OUT/gather_timing.log
b() {   # name, bench args
  local n=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { tail -20 $OUT/bench_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$n.json')); r=d.get('roofline') or {}; print('$n', d['value'], d['ms_per_step'], r.get('frac'), d.get('slice_efficiency'))"
}
b c2 --steps 5 --warmup 2
b c3 --config c3 --steps 1 --no-cpu --no-slices
b c4 --config c4 --steps 1 --no-cpu --no-slices
b c5 --config c5 --steps 2 --no-cpu --no-slices
b c1 --config c1 --steps 3 --no-cpu --no-slices
b c2_dl --integrator directlighting --strategy all --steps 2 --no-cpu --no-slices
b c3_dl --config c3 --integrator directlighting --strategy all --steps 1 --no-cpu --no-slices
b c5_dl --config c5 --integrator directlighting --strategy all --steps 1 --no-cpu --no-slices
b c2_spec --renderer spectral --steps 1 --no-cpu --no-slices
b c2_meta --integrator metadata --strategy depth --steps 3 --no-cpu --no-slices
bash tools/gpu_profile.sh r03y_c2 c2
bash tools/gpu_profile.sh r03y_dl c2 --integrator directlighting --strategy all
du -sh gpurun_out
