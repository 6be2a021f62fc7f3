#!/bin/bash
# Experiment build of libpbrtgpu.so that recompiles only the named k_shade variants with extra
# flags and links them with the product objects of every other translation unit (lib/obj, from the
# last `make`) -> lib/exp/NAME.so (timing A/B only; run with PBRTGPU_LIB=...).
# Usage: bash tools/build_exp_vars.sh NAME "32_1 32_7_dl ..." [flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; VARS=$2; shift 2
cd $R/pbrt-v2-spectral_amd
T=lib/exp/$NAME.obj; rm -rf $T; mkdir -p $T
cp lib/obj/*.o $T/
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DPGD_EXPERIMENT_BUILD -I../include -Ihost -Icsrc"
pids=()
for v in $VARS; do
  IFS=_ read nb feat dl <<< "$v"
  $H "$@" -DSHADE_NB=$nb -DSHADE_FEAT=$feat ${dl:+-DSHADE_DL=1} -c csrc/shade.hip -o $T/shade_$v.o & pids+=($!)
done
for p in ${pids[@]}; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $T/*.o -o lib/exp/$NAME.so
rm -rf $T
echo built lib/exp/$NAME.so
