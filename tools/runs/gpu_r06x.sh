#!/bin/bash
# r06x: the path integrator's MIS ray records in two sets by queue set (the drain's first
# list-mode pass overwrote records another slot had still to read) -- GPU suite, 30 renders of
# the C3 frame against its golden, then the C2 / C3 / C5 lines
OUT=$PWD/gpurun_out/r06x
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
F=bunny_frame_c3_1920x1080s1024
timeout -k 10 500 python3 tools/frame_repeat.py $F 30 > $OUT/c3rep.jsonl 2> $OUT/c3rep.err || { tail -5 $OUT/c3rep.err; exit 1; }
grep -v '"n_bad": 0' $OUT/c3rep.jsonl | cut -c1-400 || true
wc -l $OUT/c3rep.jsonl
for c in "c2 --config c2" "c3 --config c3" "c5 --config c5"; do
set -- $c; tag=$1; shift
timeout -k 10 300 python3 bench.py "$@" --no-cpu --no-slices > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag',d['value'],r['frac'],{k:v['ms_per_frame'] for k,v in r['kernels'].items()})"
done
echo done
