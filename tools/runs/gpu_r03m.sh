#!/bin/bash
# round-3 band-loop unroll A/B (C2, C3, C5) + GPU test suite
set -e
mkdir -p gpurun_out/r03m
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03m/tests.log 2>&1 || { tail -30 gpurun_out/r03m/tests.log; exit 1; }
tail -2 gpurun_out/r03m/tests.log
bash tools/gpu_exp_bench.sh r03m/c2
bash tools/gpu_exp_bench.sh r03m/c5 --config c5
bash tools/gpu_exp_bench.sh r03m/c3 --config c3 --steps 1
