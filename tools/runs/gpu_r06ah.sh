#!/bin/bash
# r06ah: C4 on FEAT_NOSPEC objects (60_22: matte / plastic / metal / substrate kinds only, 950 -> 912 KB
# of k_shade code) -- GPU suite (C4 whole frame included), then A/B against the previous library on C4
OUT=$PWD/gpurun_out/r06ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 600 bash tools/gpu_ab_rounds.sh r06ah/ab_c4 2 "--config c4" prev || exit 1
echo done
