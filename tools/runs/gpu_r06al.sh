#!/bin/bash
# r06al: the final tree's other §8 lines -- SpectralRenderer (C2, 32 wave bands), metadata (depth),
# C3 and C5 DirectLighting, and C2 over the BVH built on the GPU
OUT=$PWD/gpurun_out/r06al
mkdir -p $OUT
export TMPDIR=/tmp
for c in "spec --renderer spectral --wave-bands 32" "meta --integrator metadata" "c3dl --config c3 --integrator directlighting" "c5dl --config c5 --integrator directlighting" "bvhgpu --bvh gpu"; do
set -- $c; tag=$1; shift
timeout -k 10 600 python3 bench.py "$@" --no-cpu --no-slices > $OUT/bench_$tag.json 2> $OUT/bench_$tag.err || { tail -20 $OUT/bench_$tag.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_$tag.json'));r=d['roofline'];print('$tag',d['metric'],d['value'],d['unit'],d['ms_per_step'],r['frac'],{k:v['ms_per_frame'] for k,v in r['kernels'].items()})"
done
echo done
