#!/bin/bash
# GPU suite; C3 lookup cost split (experiment libs); DL FEAT 0 vs full variant; slice efficiency
# and per-pass log of C2; per-config rocprof profiles (trace + PMC): C3, C4, C5, C2 DL, C2
set -e
mkdir -p gpurun_out/r03o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03o/tests.log 2>&1 || { tail -30 gpurun_out/r03o/tests.log; exit 1; }
tail -2 gpurun_out/r03o/tests.log
bash tools/gpu_exp_bench.sh r03o/c3exp --config c3 --steps 1
mv pbrt-v2-spectral_amd/lib/exp pbrt-v2-spectral_amd/lib/exp.off
D="--integrator directlighting --strategy all --no-cpu --no-slices --steps 3 --warmup 1"
timeout -k 10 200 python3 bench.py $D > gpurun_out/r03o/dl_feat0.json 2> gpurun_out/r03o/dl_feat0.err
PBRTGPU_SHADE_FULL=1 timeout -k 10 200 python3 bench.py $D > gpurun_out/r03o/dl_full.json 2> gpurun_out/r03o/dl_full.err
python3 -c "
import json
for n in ('dl_feat0', 'dl_full'):
    d = json.load(open('gpurun_out/r03o/%s.json' % n)); print(n, d['value'], {k: v['ms_per_frame'] for k, v in d['roofline']['kernels'].items()})"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/r03o/c2_bench.json 2> gpurun_out/r03o/c2_bench.err
python3 -c "
import json; d = json.load(open('gpurun_out/r03o/c2_bench.json')); print('c2', d['value'], d['slice_efficiency'])"
NS=8,1 PBRTGPU_PASS_LOG=1 timeout -k 10 200 python3 tools/slice_timing.py > gpurun_out/r03o/slices.log 2> gpurun_out/r03o/passes.log
bash tools/gpu_profile.sh r03o_c3 c3
bash tools/gpu_profile.sh r03o_c4 c4
bash tools/gpu_profile.sh r03o_c5 c5
bash tools/gpu_profile.sh r03o_dl c2 --integrator directlighting --strategy all
bash tools/gpu_profile.sh r03o_c2 c2
