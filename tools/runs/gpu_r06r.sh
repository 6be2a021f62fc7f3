#!/bin/bash
# r06r: determinism of the C3 frame -- 4 renders each with the FEAT_BASIC library (32_9) and the
# previous one (32_1), tiles against the golden and pixels against the first render
OUT=$PWD/gpurun_out/r06r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/frame_repeat.py bunny_frame_c3_1920x1080s1024 4 > $OUT/cur.jsonl 2> $OUT/cur.err || { tail -5 $OUT/cur.err; exit 1; }
cat $OUT/cur.jsonl
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/prev.so timeout -k 10 200 python3 tools/frame_repeat.py bunny_frame_c3_1920x1080s1024 4 > $OUT/prev.jsonl 2> $OUT/prev.err || { tail -5 $OUT/prev.err; exit 1; }
cat $OUT/prev.jsonl
echo done
