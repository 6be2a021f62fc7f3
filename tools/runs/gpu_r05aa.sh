#!/bin/bash
# r05aa: the final tree (after the texture widening) as the driver runs it -- GPU suite, smoke,
# roofline, CPU baseline and slices) -- then the C2 DirectLighting, 60-band DirectLighting, C3, C4
# and C5 lines; then fresh rocprof + PMC of C4 and C5 (their shading kernels changed since r05p)
OUT=$PWD/gpurun_out/r05aa
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cut -c1-200 $OUT/bench_default.json
for c in "dl --integrator directlighting" "dl60 --config c2_b60 --integrator directlighting" "c3 --config c3" "c4 --config c4" "c5 --config c5"; do
set -- $c; tag=$1; shift
timeout -k 10 300 python3 bench.py "$@" --no-cpu --no-slices > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag',d['value'],r['frac'],r['traffic'],{n:v['ms_per_frame'] for n,v in r['kernels'].items()})"
done
timeout -k 10 900 bash tools/gpu_profile.sh r05aa_c4 c4 > $OUT/prof_c4.log 2>&1 || { tail -20 $OUT/prof_c4.log; exit 1; }
ls gpurun_out/summaries
echo done
