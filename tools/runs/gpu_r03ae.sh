#!/bin/bash
# one GPU's 1/4 and 1/8 of C2 and the whole frame (tools/slice_timing.py, min of 3 renders) under
# the slot rules: default (16 M target, half of the items), all items (PBRTGPU_SLOT_DIV=1), and
# round 3's first rule (PBRTGPU_SLOTS=8388608: min(items, 4 M) per lane); two interleaved rounds
set -e
OUT=$PWD/gpurun_out/r03ae
mkdir -p $OUT
for r in 1 2; do
  for s in "X=0" "PBRTGPU_SLOT_DIV=1" "PBRTGPU_SLOTS=8388608"; do
    env $s NS=4,8,1 timeout -k 10 200 python3 tools/slice_timing.py > $OUT/slices_${s}_$r.log 2>&1 || { tail -5 $OUT/slices_${s}_$r.log; exit 1; }
    echo "$s round $r: $(grep frame $OUT/slices_${s}_$r.log | sed 's/default //; s/ per GPU.*//' | tr '\n' ' ')"
  done
done
