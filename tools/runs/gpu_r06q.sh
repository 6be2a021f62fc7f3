#!/bin/bash
# r06q: timing of the FEAT_BASIC objects (r06p failed one C3 tile with 32_9) -- A/B against prev
# (FEAT 0 / FEAT_MEAS objects) and nomat (no material-switch pruning), then the GPU suite in full
OUT=$PWD/gpurun_out/r06q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06q/ab_c2 2 "--config c2" prev nomat || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06q/ab_c5 1 "--config c5" prev nomat || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06q/ab_c3 1 "--config c3" prev || exit 1
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
tail -8 $OUT/pytest_gpu.log
echo done
