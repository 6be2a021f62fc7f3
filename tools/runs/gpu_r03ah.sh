#!/bin/bash
# what the driver runs at round end, on the final tree: GPU suite, smoke, default bench line
set -e
OUT=$PWD/gpurun_out/r03ah
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -5 $OUT/smoke.log
T0=$(date +%s); timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo "bench wall: $(( $(date +%s) - T0 )) s"
