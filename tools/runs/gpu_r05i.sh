#!/bin/bash
# r05i: the final tree -- GPU suite (cylinders, the anisotropic Ward material), smoke, then
# rocprof kernel traces + PMC passes (tools/gpu_profile.sh) of C2, C2 DirectLighting, C3, C4, C5
OUT=$PWD/gpurun_out/r05i
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -3 $OUT/smoke.log
timeout -k 10 600 bash tools/gpu_profile.sh r05i_c2 c2 > $OUT/prof_c2.log 2>&1 || { tail -20 $OUT/prof_c2.log; exit 1; }
timeout -k 10 600 bash tools/gpu_profile.sh r05i_dl c2 --integrator directlighting > $OUT/prof_dl.log 2>&1 || { tail -20 $OUT/prof_dl.log; exit 1; }
timeout -k 10 900 bash tools/gpu_profile.sh r05i_c3 c3 > $OUT/prof_c3.log 2>&1 || { tail -20 $OUT/prof_c3.log; exit 1; }
timeout -k 10 900 bash tools/gpu_profile.sh r05i_c4 c4 > $OUT/prof_c4.log 2>&1 || { tail -20 $OUT/prof_c4.log; exit 1; }
timeout -k 10 600 bash tools/gpu_profile.sh r05i_c5 c5 > $OUT/prof_c5.log 2>&1 || { tail -20 $OUT/prof_c5.log; exit 1; }
ls gpurun_out/summaries
echo done
