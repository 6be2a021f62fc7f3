#!/bin/bash
# Experiment build of libpbrtgpu.so that recompiles only pbrtgpu.hip and the 32-band path shade
# variants with extra flags (the other variants are the product objects in lib/obj).
# -> pbrt-v2-spectral_amd/lib/exp/NAME.so   Usage: bash tools/build_exp1.sh NAME [flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
cd $R/pbrt-v2-spectral_amd
T=lib/exp/$NAME.obj; rm -rf $T; mkdir -p $T
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DPGD_EXPERIMENT_BUILD -I../include -Ihost -Icsrc"
$H "$@" -DSHADE_NB=32 -DSHADE_FEAT=0 -c csrc/shade.hip -o $T/s32_0.o &
p1=$!
$H "$@" -DSHADE_NB=32 -DSHADE_FEAT=7 -c csrc/shade.hip -o $T/s32_7.o &
p2=$!
$H "$@" -c csrc/pbrtgpu.hip -o $T/p.o &
p3=$!
wait $p1 $p2 $p3
others=$(ls lib/obj/shade_*.o | grep -v "shade_32_0.o\|shade_32_7.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/*.o lib/obj/lbvh.o lib/obj/loopsubdiv.o $others -o lib/exp/$NAME.so
rm -rf $T
echo built lib/exp/$NAME.so
