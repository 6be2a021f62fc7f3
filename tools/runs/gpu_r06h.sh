#!/bin/bash
# r06h: one GPU's C2 tile slices (1/8, 1/4) under slot-pool and tail settings
# (PBRTGPU_SLOT_DIV: items / d per lane when a lane has at most the slot target; PBRTGPU_TAIL: the
# queued rays at which k_tail finishes the drain) -- tools/slice_run.py, best of 3 calls each
OUT=$PWD/gpurun_out/r06h
mkdir -p $OUT
export TMPDIR=/tmp
for sl in 8 4; do
for cfg in "def" "div1 PBRTGPU_SLOT_DIV=1" "div3 PBRTGPU_SLOT_DIV=3" "tail64k PBRTGPU_TAIL=65536" "tail512k PBRTGPU_TAIL=524288" "tail1m PBRTGPU_TAIL=1048576" "def2"; do
set -- $cfg; tag=$1; shift
env "$@" timeout -k 10 120 python3 tools/slice_run.py --config c2 --slice $sl --reps 3 > $OUT/s${sl}_$tag.jsonl 2> $OUT/s${sl}_$tag.err || { tail -5 $OUT/s${sl}_$tag.err; exit 1; }
python3 -c "
import json;r=[json.loads(l) for l in open('$OUT/s${sl}_$tag.jsonl')][1:];b=min(r,key=lambda x:x['ms']);print('slice 1/$sl $tag', b['ms'], b['Mpaths_s'], b['passes'], b['gather_ms'])"
done
done
timeout -k 10 120 python3 tools/slice_run.py --config c2 --slice 1 --reps 2 > $OUT/full.jsonl 2>&1 && tail -1 $OUT/full.jsonl | cut -c1-200
echo done
