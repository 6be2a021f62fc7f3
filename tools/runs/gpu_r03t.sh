#!/bin/bash
# the drain-list GPU test, then 1/8 and full C2 frames against the lane slot rule (PBRTGPU_SLOT_DIV)
set -e
OUT=$PWD/gpurun_out/r03t
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "drain_list or unwritten" > $OUT/pytest_drain.log 2>&1 || { tail -30 $OUT/pytest_drain.log; exit 1; }
tail -1 $OUT/pytest_drain.log
for r in 1 2; do
  for dv in 4 2 1; do
    PBRTGPU_SLOT_DIV=$dv NS=8,1 timeout -k 10 200 python3 tools/slice_timing.py > $OUT/slices_div${dv}_$r.log 2>&1 || { tail -5 $OUT/slices_div${dv}_$r.log; exit 1; }
    echo "div $dv round $r: $(grep frame $OUT/slices_div${dv}_$r.log | tr '\n' ' ')"
  done
done
