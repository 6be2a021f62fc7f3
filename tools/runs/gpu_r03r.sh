#!/bin/bash
# GPU suite, then C2 with / without the drain's live-slot list (PBRTGPU_DRAIN_LIST), slices included
set -e
OUT=$PWD/gpurun_out/r03r
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  for d in 1 0; do
    PBRTGPU_DRAIN_LIST=$d timeout -k 10 200 python3 bench.py --no-cpu --steps 5 --warmup 2 > $OUT/c2_list${d}_$r.json 2> $OUT/c2_list${d}_$r.err || { tail -5 $OUT/c2_list${d}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_list${d}_$r.json')); print('list$d', $r, d['value'], d['ms_per_step'], d.get('slice_efficiency'), {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
  done
done
NS=8,1 PBRTGPU_PASS_LOG=1 timeout -k 10 200 python3 tools/slice_timing.py > $OUT/slices.log 2> $OUT/passes.log
cat $OUT/slices.log
