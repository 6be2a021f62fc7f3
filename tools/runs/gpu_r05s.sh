#!/bin/bash
# r05s: where a slice's wall time goes -- render vs host gather per call (tools/slice_run.py), 1/8
# and 1/4 and the full frame, with the pass log of one 1/8 call
OUT=$PWD/gpurun_out/r05s
mkdir -p $OUT
export TMPDIR=/tmp
for n in 8 4 1; do
timeout -k 10 200 python3 tools/slice_run.py --slice $n --reps 3 > $OUT/slice$n.jsonl 2> $OUT/slice$n.err || { tail -20 $OUT/slice$n.err; exit 1; }
cut -c1-260 $OUT/slice$n.jsonl
done
PBRTGPU_PASS_LOG=1 timeout -k 10 200 python3 tools/slice_run.py --slice 8 --reps 1 > $OUT/slice8_log.jsonl 2> $OUT/slice8_passlog.txt || { tail -20 $OUT/slice8_passlog.txt; exit 1; }
echo done
