#!/bin/bash
# GPU suite with the lane poll (hipEventQuery) and 8 passes per read-back, then C2 A/B against
# 4 passes per read-back (lib/exp/pb4), three interleaved rounds
set -e
OUT=$PWD/gpurun_out/r03w
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/gpu_ab_rounds.sh r03w_ab 3 "--steps 5 --warmup 2" pb4
