#!/bin/bash
# r06n: shape type in DevTri a.w and vcross via DFMA, tri_hit branchy as before --
# GPU suite, then A/B against the previous library
OUT=$PWD/gpurun_out/r06n
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06n/ab_c2 2 "--config c2" prev || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06n/ab_dl 1 "--config c2 --integrator directlighting" prev || exit 1
echo done
