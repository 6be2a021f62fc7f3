#!/bin/bash
# r06ae: the final tree of round 6 (after the basic DL / RGB objects) -- GPU suite + smoke, the default bench line (C2 with
# roofline, CPU baseline, slices, setup, HBM GB/s), then C3 / C5 (slices), C4, C1, and C2
# DirectLighting (32 and 60 bands); then the FEAT_BASIC k_shade forced to 4 waves/SIMD (lib/exp/w4: 128
# VGPRs, 143 spilled) against the product library on C2
OUT=$PWD/gpurun_out/r06ae
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
cp gpurun_out/frame_parity.jsonl $OUT/ 2>/dev/null; rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('c2',d['value'],r['frac'],d['setup_ms'],d['hbm_GBps'],{k:v['efficiency'] for k,v in d['slice_efficiency'].items() if k.startswith('1/')},d['cpu_baseline']['value'])"
for c in "c3 --config c3" "c5 --config c5" "c4 --config c4 --no-slices" "c1 --config c1 --no-slices" "dl --integrator directlighting --no-slices" "dl60 --config c2_b60 --integrator directlighting --no-slices"; do
set -- $c; tag=$1; shift
timeout -k 10 400 python3 bench.py "$@" --no-cpu > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];s=d.get('slice_efficiency');print('$tag',d['value'],r['frac'],d.get('hbm_GBps'),{k:v['efficiency'] for k,v in s.items() if k.startswith('1/')} if s else '')"
done
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06ae/ab_w4 2 "--config c2" w4 || exit 1
echo done
