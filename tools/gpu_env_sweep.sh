#!/bin/bash
# Timing of the product library under environment overrides (slot count etc.), one bench
# run per setting.  Usage: bash tools/gpu_env_sweep.sh TAG "VAR=val ..." ["VAR=val ..."]...
set -e
OUT=$PWD/gpurun_out/${1:-sweep}; shift
mkdir -p $OUT
i=0
for s in "$@"; do
  i=$((i+1))
  env $s timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/env$i.json
  python3 -c "import json; d=json.load(open('$OUT/env$i.json')); print('$s', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
done
