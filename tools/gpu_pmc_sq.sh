#!/bin/bash
# SQ counters of the path kernels (separate pass per counter group).  Usage: bash tools/gpu_pmc_sq.sh TAG
set -e
TAG=${1:-sq}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --res 350 --spp 64 > $OUT/b1.json 2> $OUT/p1.err
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --res 350 --spp 64 > $OUT/b2.json 2> $OUT/p2.err
echo done
