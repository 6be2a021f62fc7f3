#!/bin/bash
# Quick check + SQ stall breakdown of the path kernels.  Usage: bash tools/gpu_sq.sh TAG
set -e
TAG=${1:-sq}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['roofline']['kernel_ms_per_step'])"
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -o -E "(SQC?|TCP|TCC|TA|TD)_[A-Z0-9_]*(ICACHE|IFETCH|INST_LEVEL|LEVEL_WAVES|INSTS_SMEM|WAIT_INST)[A-Z0-9_]*" $OUT/counters.txt | sort -u > $OUT/ic_counters.txt || true
cat $OUT/ic_counters.txt | tr '\n' ' '; echo
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $OUT/p1 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --res 350 --spp 64 > $OUT/b1.json 2> $OUT/p1.err
echo done
