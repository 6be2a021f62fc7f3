#!/bin/bash
# Cache-hierarchy counters of the path kernels (one rocprofv3 pass per counter group).
# Usage: bash tools/gpu_pmc_mem.sh TAG [bench args]
set -e
TAG=${1:-mem}; shift || true
ARGS=${@:---res 350 --spp 64}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ TCP_TCC_READ_REQ_LATENCY TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES GRBM_GUI_ACTIVE -d $OUT/m1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu $ARGS > $OUT/m1.json 2> $OUT/m1.err
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_READ TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS -d $OUT/m2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu $ARGS > $OUT/m2.json 2> $OUT/m2.err
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $OUT/m3 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu $ARGS > $OUT/m3.json 2> $OUT/m3.err
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVE_CYCLES -d $OUT/m4 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu $ARGS > $OUT/m4.json 2> $OUT/m4.err
echo done
