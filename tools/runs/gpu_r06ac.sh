#!/bin/bash
# r06ac: one GPU's C2 1/8 and 1/4 tile slices under the read-back batch sizes of the drain
# (PBRTGPU_DRAIN_BATCH, default 2) and of the last slot pool before it (PBRTGPU_NEAR_BATCH, default
# 4) -- tools/slice_run.py, best of 3 calls each
OUT=$PWD/gpurun_out/r06ac
mkdir -p $OUT
export TMPDIR=/tmp
for sl in 8 4; do
for cfg in "def" "d1 PBRTGPU_DRAIN_BATCH=1" "d4 PBRTGPU_DRAIN_BATCH=4" "n2 PBRTGPU_NEAR_BATCH=2" "n8 PBRTGPU_NEAR_BATCH=8" "d4n8 PBRTGPU_DRAIN_BATCH=4 PBRTGPU_NEAR_BATCH=8" "d1n2 PBRTGPU_DRAIN_BATCH=1 PBRTGPU_NEAR_BATCH=2" "def2"; do
set -- $cfg; tag=$1; shift
env "$@" timeout -k 10 120 python3 tools/slice_run.py --config c2 --slice $sl --reps 3 > $OUT/s${sl}_$tag.jsonl 2> $OUT/s${sl}_$tag.err || { tail -5 $OUT/s${sl}_$tag.err; exit 1; }
python3 -c "
import json;r=[json.loads(l) for l in open('$OUT/s${sl}_$tag.jsonl')][1:];b=min(r,key=lambda x:x['ms']);print('slice 1/$sl $tag', b['ms'], b['Mpaths_s'], b['passes'], b['gather_ms'])"
done
done
for cfg in "def" "d4n8 PBRTGPU_DRAIN_BATCH=4 PBRTGPU_NEAR_BATCH=8" "d1 PBRTGPU_DRAIN_BATCH=1"; do
set -- $cfg; tag=$1; shift
env "$@" timeout -k 10 120 python3 tools/slice_run.py --config c2 --slice 1 --reps 2 > $OUT/full_$tag.jsonl 2> $OUT/full_$tag.err || { tail -5 $OUT/full_$tag.err; exit 1; }
python3 -c "
import json;r=[json.loads(l) for l in open('$OUT/full_$tag.jsonl')][1:];b=min(r,key=lambda x:x['ms']);print('full $tag', b['ms'], b['Mpaths_s'], b['passes'])"
done
echo done
