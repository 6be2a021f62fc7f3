#!/bin/bash
# r05o: the lanes staggered by one shade pass (PBRTGPU_LANE_STAGGER=1) against in-step lanes:
# C2 full frame and slices, interleaved
OUT=$PWD/gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
for m in 0 1 0 1; do
PBRTGPU_LANE_STAGGER=$m timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench_c2_s$m.json 2> $OUT/bench_c2_s$m.err || { tail -20 $OUT/bench_c2_s$m.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c2_s$m.json'));s=d['slice_efficiency'];print('stagger=$m',d['value'],[(k,s[k]['efficiency'],s[k]['ms']) for k in ('1/2','1/4','1/8')])"
done
echo done
