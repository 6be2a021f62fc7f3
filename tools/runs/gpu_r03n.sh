#!/bin/bash
# measured-BRDF lookup: final radius first vs the retry loop (C3) + the GPU test suite
set -e
mkdir -p gpurun_out/r03n
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03n/tests.log 2>&1 || { tail -30 gpurun_out/r03n/tests.log; exit 1; }
tail -2 gpurun_out/r03n/tests.log
bash tools/gpu_exp_bench.sh r03n/c3 --config c3 --steps 1
