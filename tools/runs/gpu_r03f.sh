#!/bin/bash
set -e
OUT=$PWD/gpurun_out/r03f
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/gpu_exp_bench.sh r03f/c2
bash tools/gpu_exp_bench.sh r03f/dl --integrator directlighting --strategy all
