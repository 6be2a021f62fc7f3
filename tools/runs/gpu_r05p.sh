#!/bin/bash
# r05p: rocprof kernel traces + PMC passes (tools/gpu_profile.sh) of the current tree: C3 (the
# FEAT_MEAS build), C4 (the 60-band TEX|INF build), C2 DirectLighting, C2, C5
OUT=$PWD/gpurun_out/r05p
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 bash tools/gpu_profile.sh r05p_c3 c3 > $OUT/prof_c3.log 2>&1 || { tail -20 $OUT/prof_c3.log; exit 1; }
timeout -k 10 900 bash tools/gpu_profile.sh r05p_c4 c4 > $OUT/prof_c4.log 2>&1 || { tail -20 $OUT/prof_c4.log; exit 1; }
timeout -k 10 600 bash tools/gpu_profile.sh r05p_dl c2 --integrator directlighting > $OUT/prof_dl.log 2>&1 || { tail -20 $OUT/prof_dl.log; exit 1; }
timeout -k 10 600 bash tools/gpu_profile.sh r05p_c2 c2 > $OUT/prof_c2.log 2>&1 || { tail -20 $OUT/prof_c2.log; exit 1; }
timeout -k 10 600 bash tools/gpu_profile.sh r05p_c5 c5 > $OUT/prof_c5.log 2>&1 || { tail -20 $OUT/prof_c5.log; exit 1; }
ls gpurun_out/summaries
echo done
