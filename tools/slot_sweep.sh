#!/bin/bash
# GPU-box experiment: C2 frame rate against the path-slot pool size (PBRTGPU_SLOTS, split over
# two lanes).  Usage (repo root, GPU box): bash tools/slot_sweep.sh TAG [bench args]
TAG=${1:-sweep}
shift || true
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
for S in 8388608 2097152 1048576 524288 262144; do
  PBRTGPU_SLOTS=$S timeout -k 10 120 python3 bench.py --no-cpu --no-roofline --steps 2 --warmup 1 "$@" > $OUT/slots_$S.json 2> $OUT/slots_$S.err || exit 1
  echo "$S $(python3 -c "import json,sys; d=json.load(open('$OUT/slots_$S.json')); print(d['value'], d['ms_per_step'])")"
done
