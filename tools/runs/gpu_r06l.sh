#!/bin/bash
# r06l: the traversal kernels' child-box tests straight-line (slab_enter_bf) and the 4-wide closest
# walk's slot picks as bit selects -- GPU suite (intersect KAT, goldens, frames), then A/B against
# the previous library (lib/exp/prev) on C2, C5 and C2 DirectLighting
OUT=$PWD/gpurun_out/r06l
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06l/ab_c2 3 "--config c2" prev || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06l/ab_c5 2 "--config c5" prev || exit 1
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06l/ab_dl 2 "--config c2 --integrator directlighting" prev || exit 1
echo done
