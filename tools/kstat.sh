#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy / code bytes of the gfx950 device code, for the
# given extra -D flags.  Usage: bash tools/kstat.sh [-DFLAG ...]
# (SHADE_VAR=nb_feat selects the k_shade variant compiled beside pbrtgpu.hip; default 32_0)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
V=${SHADE_VAR:-32_0}
: > $T/rem.txt; : > $T/sizes.txt
for SRC in pbrtgpu.hip shade.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DSHADE_NB=${V%_*} -DSHADE_FEAT=${V#*_} "$@" \
    -I$R/include -I$R/pbrt-v2-spectral_amd/host -I$R/pbrt-v2-spectral_amd/csrc --cuda-device-only \
    -c $R/pbrt-v2-spectral_amd/csrc/$SRC -o $T/dev.co -Rpass-analysis=kernel-resource-usage 2>> $T/rem.txt
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input=$T/dev.co --output=$T/dev.elf \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --unbundle
  /opt/rocm/lib/llvm/bin/llvm-readelf -s $T/dev.elf | awk '$4=="FUNC"{print $8, $3}' >> $T/sizes.txt
done
sort -u -o $T/sizes.txt $T/sizes.txt
grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" $T/rem.txt | sed 's/.*remark: //; s/ \[-Rpass.*//' | paste - - - - |
  awk -F'\t' '{n=$1; sub(/Function Name: /,"",n); v=$2; sub(/.*: /,"",v); s=$3; sub(/.*: /,"",s); o=$4; sub(/.*: /,"",o); print n, v, s, o}' |
  sort -u > $T/res.txt
join $T/res.txt $T/sizes.txt | awk '{printf "%-70s vgpr %4s scratch %4s occ %s code %8d\n", substr($1,1,70), $2, $3, $4, $5}'
rm -rf $T
