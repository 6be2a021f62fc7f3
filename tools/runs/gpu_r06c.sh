#!/bin/bash
# r06c: per-primitive shading records + pipelined batches (hybrid) -- GPU suite (C1 + C3 frames),
# A/B of the records (lib/exp/norec: the prim -> triangle -> vertex chain) on C2 and C3, then the
# three pipeline modes (PBRTGPU_PIPE=0/1/2) on the C2 line with its slices
OUT=$PWD/gpurun_out/r06c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
cp gpurun_out/frame_parity.jsonl $OUT/ 2>/dev/null; rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 900 bash tools/gpu_ab_rounds.sh r06c/ab_c2 3 "--config c2" norec || exit 1
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06c/ab_c3 2 "--config c3 --steps 2" norec || exit 1
for p in 0 1 2 0 1 2; do
PBRTGPU_PIPE=$p timeout -k 10 300 python3 bench.py --no-cpu > $OUT/pipe$p.json 2> $OUT/pipe$p.err || { tail -20 $OUT/pipe$p.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/pipe$p.json'));r=d['roofline'];print('pipe $p',d['value'],r['frac'],{k:v['efficiency'] for k,v in d['slice_efficiency'].items() if k.startswith('1/')})"
done
echo done
