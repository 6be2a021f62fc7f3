#!/bin/bash
# GPU-box round check: parity tests, smoke, then bench on each config.
# Usage: bash tools/gpu_round.sh TAG [configs...]   (default configs: c2 c3 c4 c5)
set -e
TAG=${1:-round}
shift || true
CFGS=${@:-c2 c3 c4 c5}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for c in $CFGS; do
  if [ $c = c2 ]; then EXTRA=""; else EXTRA="--steps 1 --no-cpu"; fi
  timeout -k 10 300 python3 bench.py --config $c $EXTRA > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  cat $OUT/bench_$c.json
done
