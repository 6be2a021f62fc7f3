#!/bin/bash
# GPU box: serial-mode kernel traces of one bench command with the current library and with
# experiment libraries lib/exp/NAME.so (PBRTGPU_LIB).  Usage: bash tools/gpu_ab_trace.sh TAG "bench args" NAME...
set -e
TAG=$1; ARGS=$2; shift 2
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for e in cur "$@"; do
  L=""; [ $e != cur ] && L=$PWD/pbrt-v2-spectral_amd/lib/exp/$e.so
  PBRTGPU_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$e -o run -- python3 bench.py --no-cpu --no-roofline --steps 1 --warmup 1 --serial $ARGS > $OUT/$e.json 2> $OUT/$e.err
  python3 -c "import json; d=json.load(open('$OUT/$e.json')); print('$e', d['value'], d['ms_per_step'])"
done
