#!/bin/bash
# r06v: is the C3 frame's rare one-pixel difference a sample no path wrote? -- 20 renders with
# PBRTGPU_POISON=255 (slot arrays and the per-sample radiance buffer NaN before each batch): an
# unwritten sample shows as a non-finite pixel
OUT=$PWD/gpurun_out/r06v
mkdir -p $OUT
export TMPDIR=/tmp
F=bunny_frame_c3_1920x1080s1024
PBRTGPU_POISON=255 timeout -k 10 400 python3 tools/frame_repeat.py $F 20 > $OUT/poison.jsonl 2> $OUT/poison.err || { tail -5 $OUT/poison.err; exit 1; }
grep -v '"n_bad": 0' $OUT/poison.jsonl | cut -c1-700 || true
wc -l $OUT/*.jsonl
echo done
