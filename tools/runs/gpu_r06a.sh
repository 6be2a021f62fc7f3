#!/bin/bash
# r06a: round-6 baseline of the round-5 final tree -- default bench line (C2: roofline, CPU
# baseline, slices, setup, HBM GB/s), then C3 and C5 with their slice_efficiency blocks
OUT=$PWD/gpurun_out/r06a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cut -c1-300 $OUT/bench_default.json
for c in "c3 --config c3" "c5 --config c5"; do
set -- $c; tag=$1; shift
timeout -k 10 400 python3 bench.py "$@" --no-cpu > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag',d['value'],r['frac'],d.get('setup_ms'),d.get('hbm_GBps'),{k:v['efficiency'] for k,v in d['slice_efficiency'].items() if k.startswith('1/')})"
done
echo done
