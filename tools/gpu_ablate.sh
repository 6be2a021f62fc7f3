#!/bin/bash
# Timing ablations (experiment libraries under pbrt-v2-spectral_amd/lib/exp; not the product).
set -e
OUT=$PWD/gpurun_out/${1:-abl}
mkdir -p $OUT
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/base.json
shopt -s nullglob
for v in pbrt-v2-spectral_amd/lib/exp/*.so; do
  n=$(basename $v .so)
  PBRTGPU_LIB=$PWD/$v timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/$n.json
done
for f in $OUT/*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f'.split('/')[-1], d['value'], d['roofline']['kernel_ms_per_step'])"; done
