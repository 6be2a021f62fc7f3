#!/bin/bash
# r06i: the kd lookup's and quadric_hit's pointers in the global address space (no flat accesses in
# the out-of-line functions of the shading kernels) -- GPU suite, then A/B against the previous
# product library (lib/exp/flat) on C3, C2 and C2 DirectLighting
OUT=$PWD/gpurun_out/r06i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06i/ab_c3 3 "--config c3 --steps 2" flat || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06i/ab_c2 3 "--config c2" flat || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06i/ab_dl 2 "--config c2 --integrator directlighting" flat || exit 1
echo done
