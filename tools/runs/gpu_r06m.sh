#!/bin/bash
# r06m: shape type in DevTri a.w (one dependent load per triangle test), tri_hit straight-line,
# vcross products via DFMA (same bits) -- GPU suite, then A/B against the previous library
OUT=$PWD/gpurun_out/r06m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06m/ab_c2 3 "--config c2" prev || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06m/ab_c5 2 "--config c5" prev || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06m/ab_dl 2 "--config c2 --integrator directlighting" prev || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06m/ab_c3 1 "--config c3" prev || exit 1
echo done
