#!/bin/bash
# r06ab: FEAT_BASIC objects for 60-band DirectLighting (60_8_dl) and the RGB build's path
# integrator (3_8, C1) -- GPU suite, then A/B against the previous library on C2's scene at 60
# bands with DirectLighting and on C1
OUT=$PWD/gpurun_out/r06ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06ab/ab_dl60 2 "--config c2_b60 --integrator directlighting" prev || exit 1
timeout -k 10 300 bash tools/gpu_ab_rounds.sh r06ab/ab_c1 3 "--config c1" prev || exit 1
echo done
