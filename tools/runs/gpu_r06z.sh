#!/bin/bash
# r06z: DirectLighting on FEAT_BASIC objects (32_8_dl) -- GPU suite, A/B against the previous
# library (prev: FEAT 0 DL objects) on C2 DirectLighting, then rocprof + PMC of C2 DirectLighting
# and C4 (tools/gpu_profile.sh)
OUT=$PWD/gpurun_out/r06z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06z/ab_dl 2 "--config c2 --integrator directlighting" prev || exit 1
timeout -k 10 600 bash tools/gpu_profile.sh r06z_dl c2 --integrator directlighting > $OUT/prof_dl.log 2>&1 || { tail -20 $OUT/prof_dl.log; exit 1; }
timeout -k 10 700 bash tools/gpu_profile.sh r06z_c4 c4 > $OUT/prof_c4.log 2>&1 || { tail -20 $OUT/prof_c4.log; exit 1; }
ls gpurun_out/summaries
echo done
