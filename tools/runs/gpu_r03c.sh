#!/bin/bash
set -e
OUT=$PWD/gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/gpu_ab_trace.sh r03c/dl "--integrator directlighting --strategy all" prev
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c2.json')); print('path c2', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
