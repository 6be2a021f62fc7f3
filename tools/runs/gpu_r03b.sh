#!/bin/bash
# round-3 check: GPU suite, DirectLighting (k_dl_spec split) and path benches
set -e
OUT=$PWD/gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu --integrator directlighting --strategy all > $OUT/dl_c2.json 2> $OUT/dl_c2.err || { tail -20 $OUT/dl_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/dl_c2.json')); print('DL c2', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > $OUT/c2.json 2> $OUT/c2.err || { tail -20 $OUT/c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/c2.json')); print('path c2', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
