#!/bin/bash
# r06t: the C3 frame's rare one-pixel difference -- 20 renders each: defaults, one serial lane
# (PBRTGPU_SERIAL=1) and the kd-trees read from global memory (PBRTGPU_KD_LDS=0); the differing
# pixel's bands against a render that matches the golden
OUT=$PWD/gpurun_out/r06t
mkdir -p $OUT
export TMPDIR=/tmp
F=bunny_frame_c3_1920x1080s1024
timeout -k 10 300 python3 tools/frame_repeat.py $F 20 > $OUT/def.jsonl 2> $OUT/def.err || { tail -5 $OUT/def.err; exit 1; }
grep -v '"n_bad": 0' $OUT/def.jsonl | cut -c1-600 || true
PBRTGPU_SERIAL=1 timeout -k 10 300 python3 tools/frame_repeat.py $F 16 > $OUT/serial.jsonl 2> $OUT/serial.err || { tail -5 $OUT/serial.err; exit 1; }
grep -v '"n_bad": 0' $OUT/serial.jsonl | cut -c1-600 || true
PBRTGPU_KD_LDS=0 timeout -k 10 300 python3 tools/frame_repeat.py $F 16 > $OUT/kdglob.jsonl 2> $OUT/kdglob.err || { tail -5 $OUT/kdglob.err; exit 1; }
grep -v '"n_bad": 0' $OUT/kdglob.jsonl | cut -c1-600 || true
wc -l $OUT/*.jsonl
echo done
