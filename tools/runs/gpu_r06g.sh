#!/bin/bash
# r06g: C2 with the transcendentals inlined (lib/exp/tinl: all; lib/exp/thot: sincosf / powf /
# acosf / sinf only -- out-of-line calls wait for every outstanding load and store at entry);
# C3 with the kd-walk candidates in registers (lib/exp/kdreg) against the memory list (kdmem, and the
# product library)
OUT=$PWD/gpurun_out/r06g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 bash tools/gpu_ab_rounds.sh r06g/ab_c2 3 "--config c2" tinl thot || exit 1
timeout -k 10 700 bash tools/gpu_ab_rounds.sh r06g/ab_c3 2 "--config c3 --steps 2" kdmem kdreg || exit 1
echo done
