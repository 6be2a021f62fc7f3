#!/bin/bash
# r06w: more statistics on the C3 frame's rare one-pixel difference -- 40 renders with
# PBRTGPU_POISON=255 (an unwritten sample or slot read shows as non-finite), then 20 default
OUT=$PWD/gpurun_out/r06w
mkdir -p $OUT
export TMPDIR=/tmp
F=bunny_frame_c3_1920x1080s1024
PBRTGPU_POISON=255 timeout -k 10 500 python3 tools/frame_repeat.py $F 40 > $OUT/poison.jsonl 2> $OUT/poison.err || { tail -5 $OUT/poison.err; exit 1; }
grep -v '"n_bad": 0' $OUT/poison.jsonl | cut -c1-700 || true
timeout -k 10 300 python3 tools/frame_repeat.py $F 20 > $OUT/def.jsonl 2> $OUT/def.err || { tail -5 $OUT/def.err; exit 1; }
grep -v '"n_bad": 0' $OUT/def.jsonl | cut -c1-700 || true
wc -l $OUT/*.jsonl
echo done
