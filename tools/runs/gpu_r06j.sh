#!/bin/bash
# r06j: C3 with the kd walk's step as value selects (lib/exp/kdsel) against the product library
OUT=$PWD/gpurun_out/r06j
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 bash tools/gpu_ab_rounds.sh r06j/ab_c3 3 "--config c3 --steps 2" kdsel || exit 1
echo done
