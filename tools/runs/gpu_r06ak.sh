#!/bin/bash
# r06ak: rocprof + PMC of C4 on its FEAT_NOSPEC objects (the final tree; tools/gpu_profile.sh)
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ak
timeout -k 10 700 bash tools/gpu_profile.sh r06ak_c4 c4 > gpurun_out/r06ak/prof_c4.log 2>&1 || { tail -20 gpurun_out/r06ak/prof_c4.log; exit 1; }
ls gpurun_out/summaries
echo done
