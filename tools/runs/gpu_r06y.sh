#!/bin/bash
# r06y: rocprofv3 kernel trace + stats and the PMC passes (FETCH / WRITE / SQ / LDS / TCC) of the
# final tree's C2, C3 and C5 (tools/gpu_profile.sh); summaries and HBM traffic to gpurun_out/summaries
export TMPDIR=/tmp
mkdir -p gpurun_out/r06y
timeout -k 10 500 bash tools/gpu_profile.sh r06y_c2 c2 > gpurun_out/r06y/prof_c2.log 2>&1 || { tail -20 gpurun_out/r06y/prof_c2.log; exit 1; }
timeout -k 10 700 bash tools/gpu_profile.sh r06y_c3 c3 > gpurun_out/r06y/prof_c3.log 2>&1 || { tail -20 gpurun_out/r06y/prof_c3.log; exit 1; }
timeout -k 10 500 bash tools/gpu_profile.sh r06y_c5 c5 > gpurun_out/r06y/prof_c5.log 2>&1 || { tail -20 gpurun_out/r06y/prof_c5.log; exit 1; }
ls gpurun_out/summaries
echo done
