#!/bin/bash
# r06b: two batches of passes in flight per lane (run_wavefront) -- GPU suite (C1 frame added),
# then the default bench line and the C3 / C5 lines with their slices
OUT=$PWD/gpurun_out/r06b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
cp gpurun_out/frame_parity.jsonl $OUT/ 2>/dev/null; rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('c2',d['value'],r['frac'],{k:v['efficiency'] for k,v in d['slice_efficiency'].items() if k.startswith('1/')})"
for c in "c3 --config c3" "c5 --config c5"; do
set -- $c; tag=$1; shift
timeout -k 10 400 python3 bench.py "$@" --no-cpu > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag',d['value'],r['frac'],{k:v['efficiency'] for k,v in d['slice_efficiency'].items() if k.startswith('1/')})"
done
echo done
