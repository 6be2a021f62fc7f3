#!/bin/bash
# r05t: k_dl_nee at 3 waves/SIMD (experiment library lib/exp/nee3.so) against the product's 2
OUT=$PWD/gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp
for m in 0 1 0 1; do
if [ $m = 1 ]; then export PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/nee3.so; else unset PBRTGPU_LIB; fi
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl_m$m.json 2> $OUT/bench_dl_m$m.err || { tail -20 $OUT/bench_dl_m$m.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_dl_m$m.json'));k=d['roofline']['kernels'];print('nee3=$m',d['value'],k['k_shade']['ms_per_frame'])"
done
unset PBRTGPU_LIB
echo done
