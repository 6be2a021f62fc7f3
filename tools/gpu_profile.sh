#!/bin/bash
# GPU-box recipe: parity tests, smoke, bench, rocprofv3 kernel trace + PMC passes.
# Usage (from the repo root, on the GPU box): bash tools/gpu_profile.sh TAG
set -e
TAG=${1:-r01}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/bench_pmc1.json 2> $OUT/pmc1.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $OUT/bench_pmc2.json 2> $OUT/pmc2.err
echo done
