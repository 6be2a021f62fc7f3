#!/bin/bash
# r06s: where the C3 frame's rare one-pixel nondeterminism comes from -- 6 renders each with the
# defaults, without the drain's tail kernel (PBRTGPU_TAIL=0) and without the drain list
# (PBRTGPU_DRAIN_LIST=0, no tail either)
OUT=$PWD/gpurun_out/r06s
mkdir -p $OUT
export TMPDIR=/tmp
F=bunny_frame_c3_1920x1080s1024
timeout -k 10 200 python3 tools/frame_repeat.py $F 6 > $OUT/def.jsonl 2> $OUT/def.err || { tail -5 $OUT/def.err; exit 1; }
cut -c1-220 $OUT/def.jsonl
PBRTGPU_TAIL=0 timeout -k 10 200 python3 tools/frame_repeat.py $F 6 > $OUT/notail.jsonl 2> $OUT/notail.err || { tail -5 $OUT/notail.err; exit 1; }
cut -c1-220 $OUT/notail.jsonl
PBRTGPU_DRAIN_LIST=0 timeout -k 10 200 python3 tools/frame_repeat.py $F 6 > $OUT/nolist.jsonl 2> $OUT/nolist.err || { tail -5 $OUT/nolist.err; exit 1; }
cut -c1-220 $OUT/nolist.jsonl
echo done
