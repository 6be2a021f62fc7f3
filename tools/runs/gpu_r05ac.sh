#!/bin/bash
# r05ac: the final tree after the marble texture -- default bench line (roofline, CPU
# baseline, slices) then the C2 DirectLighting, 60-band DirectLighting, C3, C4 and C5 lines
OUT=$PWD/gpurun_out/r05ac
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cut -c1-200 $OUT/bench_default.json
for c in "dl --integrator directlighting" "dl60 --config c2_b60 --integrator directlighting" "c3 --config c3" "c4 --config c4" "c5 --config c5"; do
set -- $c; tag=$1; shift
timeout -k 10 300 python3 bench.py "$@" --no-cpu --no-slices > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag',d['value'],r['frac'],r['traffic'],{n:v['ms_per_frame'] for n,v in r['kernels'].items()})"
done
echo done
