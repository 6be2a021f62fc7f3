#!/bin/bash
# PC sampling of the path kernels (host-trap, time based).  Usage: bash tools/gpu_pcsample.sh TAG
set -e
TAG=${1:-pcs}
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 --output-format csv -d $OUT/pcs -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --res 350 --spp 32 > $OUT/b.json 2> $OUT/pcs.err
echo done
ls -R $OUT | head -20
