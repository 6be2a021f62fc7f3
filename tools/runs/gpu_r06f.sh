#!/bin/bash
# r06f: light 0 as a compile-time constant (lib/exp/light0, exact for C2's one light: its record,
# shapes and quadric through scalar loads) against the product library, C2, three rounds
OUT=$PWD/gpurun_out/r06f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 bash tools/gpu_ab_rounds.sh r06f/ab_c2 3 "--config c2" light0 || exit 1
echo done
