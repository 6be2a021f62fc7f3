#!/bin/bash
# C2 under environment overrides: ray-replacement threshold (PBRTGPU_REFILL) and slot target
# (PBRTGPU_SLOTS), two interleaved rounds on one box
set -e
OUT=$PWD/gpurun_out/r03aa
mkdir -p $OUT
for r in 1 2; do
  i=0
  for s in "X=0" "PBRTGPU_REFILL=8" "PBRTGPU_REFILL=24" "PBRTGPU_REFILL=32" "PBRTGPU_SLOTS=12582912" "PBRTGPU_SLOTS=16777216"; do
    i=$((i+1))
    env $s timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-slices --no-roofline > $OUT/env${i}_$r.json 2> $OUT/env${i}_$r.err || { tail -5 $OUT/env${i}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/env${i}_$r.json')); print('$s', $r, d['value'], d['ms_per_step'])"
  done
done
