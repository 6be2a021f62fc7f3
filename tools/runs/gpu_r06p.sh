#!/bin/bash
# r06p: FEAT_BASIC shading objects (matte / plastic, + measured for C3) for C2, C5 (32_8) and C3
# (32_9) -- GPU suite, then A/B against the previous library (prev: FEAT 0 / FEAT_MEAS objects) and
# the variant without the material-switch pruning (nomat)
OUT=$PWD/gpurun_out/r06p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06p/ab_c2 2 "--config c2" prev nomat || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06p/ab_c5 1 "--config c5" prev nomat || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06p/ab_c3 1 "--config c3" prev || exit 1
echo done
