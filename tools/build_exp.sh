#!/bin/bash
# Experiment build of libpbrtgpu.so with extra compile flags -> pbrt-v2-spectral_amd/lib/exp/NAME.so
# (timing ablations only; run with PBRTGPU_LIB=...).  Usage: bash tools/build_exp.sh NAME [flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
cd $R/pbrt-v2-spectral_amd
T=lib/exp/$NAME.obj; mkdir -p $T
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DPGD_EXPERIMENT_BUILD -I../include -Ihost -Icsrc"
pids=()
for v in 32_0 32_1 32_7 60_0 60_6 60_7 30_0 30_7 3_0 3_7; do
  $H "$@" -DSHADE_NB=${v%_*} -DSHADE_FEAT=${v#*_} -c csrc/shade.hip -o $T/s$v.o & pids+=($!)
  $H "$@" -DSHADE_NB=${v%_*} -DSHADE_FEAT=${v#*_} -DSHADE_DL=1 -c csrc/shade.hip -o $T/d$v.o & pids+=($!)
done
$H "$@" -c csrc/pbrtgpu.hip -o $T/p.o & pids+=($!)
$H "$@" -c csrc/lbvh.hip -o $T/lbvh.o & pids+=($!)
$H "$@" -c csrc/loopsubdiv.hip -o $T/loop.o & pids+=($!)
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/*.o -o lib/exp/$NAME.so
rm -rf $T
echo built lib/exp/$NAME.so
