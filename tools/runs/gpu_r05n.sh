#!/bin/bash
# r05n: DirectLighting without the light-sample vertex's unused differentials (FEAT 0), and C4 on a
# 60-band textures + environment-light build (no kd-tree walk) against the all-features build
OUT=$PWD/gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl_$i.json 2> $OUT/bench_dl_$i.err || { tail -20 $OUT/bench_dl_$i.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_dl_$i.json'));k=d['roofline']['kernels'];print('dl',d['value'],k['k_shade']['ms_per_frame'])"
done
for m in 0 1 0 1; do
if [ $m = 1 ]; then export PGD_NO60_6=1; else unset PGD_NO60_6; fi
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-slices > $OUT/bench_c4_n$m.json 2> $OUT/bench_c4_n$m.err || { tail -20 $OUT/bench_c4_n$m.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c4_n$m.json'));k=d['roofline']['kernels'];print('c4 no60_6=$m',d['value'],k['k_shade']['ms_per_frame'])"
done
unset PGD_NO60_6
echo done
