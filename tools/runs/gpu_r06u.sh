#!/bin/bash
# r06u: is the C3 frame's rare one-pixel difference one event per sample batch or per path? --
# 120 renders at 64 spp (one batch: the full frame's first) and 40 at 128 spp (two), pixels
# against the first render
OUT=$PWD/gpurun_out/r06u
mkdir -p $OUT
export TMPDIR=/tmp
F=bunny_frame_c3_1920x1080s1024
timeout -k 10 400 python3 tools/frame_repeat.py $F 120 64 > $OUT/s64.jsonl 2> $OUT/s64.err || { tail -5 $OUT/s64.err; exit 1; }
grep -v '"n_pix_diff": 0' $OUT/s64.jsonl | cut -c1-300 || true
timeout -k 10 400 python3 tools/frame_repeat.py $F 40 128 > $OUT/s128.jsonl 2> $OUT/s128.err || { tail -5 $OUT/s128.err; exit 1; }
grep -v '"n_pix_diff": 0' $OUT/s128.jsonl | cut -c1-300 || true
wc -l $OUT/*.jsonl
echo done
