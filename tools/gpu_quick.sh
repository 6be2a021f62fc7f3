#!/bin/bash
# GPU-box quick check: parity tests + short bench.  Usage: bash tools/gpu_quick.sh TAG [bench args...]
set -e
TAG=${1:-quick}
shift || true
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
