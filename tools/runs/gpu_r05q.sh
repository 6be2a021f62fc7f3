#!/bin/bash
# r05q: C5 with the AnimatedTransform scale factor inverted directly when diagonal (the path's
# instance matrices at path start); GPU suite first
OUT=$PWD/gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --config c5 --no-cpu --no-slices > $OUT/bench_c5_$i.json 2> $OUT/bench_c5_$i.err || { tail -20 $OUT/bench_c5_$i.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c5_$i.json'));k=d['roofline']['kernels'];print('c5',d['value'],{n:v['ms_per_frame'] for n,v in k.items()})"
done
echo done
