#!/bin/bash
# C2 with slices: slot target 8 M (default) vs 16 M (PBRTGPU_SLOTS), C4 likewise; two interleaved rounds
set -e
OUT=$PWD/gpurun_out/r03ac
mkdir -p $OUT
for r in 1 2; do
  for s in 8388608 16777216; do
    PBRTGPU_SLOTS=$s timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu --no-roofline > $OUT/c2_${s}_${r}.json 2> $OUT/c2_${s}_${r}.err || { tail -5 $OUT/c2_${s}_${r}.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c2_${s}_${r}.json')); print('c2 slots $s', $r, d['value'], d['ms_per_step'], {k: (v['efficiency'], v['passes'], v['Mpaths_s']) for k, v in d['slice_efficiency'].items() if isinstance(v, dict)})"
    PBRTGPU_SLOTS=$s timeout -k 10 300 python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu --no-roofline --no-slices > $OUT/c4_${s}_${r}.json 2> $OUT/c4_${s}_${r}.err || { tail -5 $OUT/c4_${s}_${r}.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/c4_${s}_${r}.json')); print('c4 slots $s', $r, d['value'], d['ms_per_step'])"
  done
done
