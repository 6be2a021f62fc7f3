#!/bin/bash
# r06ag: the 60-band FEAT_BASIC k_dl_spec at 2 waves/SIMD (lib/exp/spec2: 256 VGPRs, 52 spilled)
# against the product library (1 wave, 280 VGPRs) -- its basic-objects test on the experiment
# library, then A/B on C2's scene at 60 bands with DirectLighting, two rounds
OUT=$PWD/gpurun_out/r06ag
mkdir -p $OUT
export TMPDIR=/tmp
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/spec2.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "basic_material" --timeout 200 --timeout-method thread > $OUT/pytest_spec2.log 2>&1 || { tail -30 $OUT/pytest_spec2.log; exit 1; }
tail -1 $OUT/pytest_spec2.log
timeout -k 10 500 bash tools/gpu_ab_rounds.sh r06ag/ab_dl60 2 "--config c2_b60 --integrator directlighting" spec2 || exit 1
echo done
