#!/bin/bash
# r05c: GPU suite (textured material parameters: two textured spectra, textured floats, raw metal
# eta / k; the drain's tail kernel); the tail threshold on C2 (full frame and slices); where a 1/8
# slice's wall time goes (device timeline, tail off / on); the band-count experiment (k_shade at
# 16 bands on the 32-band scene vs the same build at 32)
OUT=$PWD/gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for t in 0 65536 262144 1048576; do
  PBRTGPU_TAIL=$t timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench_c2_tail$t.json 2> $OUT/bench_c2_tail$t.err || { tail -20 $OUT/bench_c2_tail$t.err; exit 1; }
  cut -c1-200 $OUT/bench_c2_tail$t.json
done
for t in 0 262144; do
  PBRTGPU_TAIL=$t timeout -k 10 200 rocprofv3 --kernel-trace -d $OUT/tl_$t -o run -- python3 tools/slice_run.py --slice 8 --reps 2 > $OUT/slice8_tail$t.jsonl 2> $OUT/slice8_tail$t.err || { tail -20 $OUT/slice8_tail$t.err; exit 1; }
  cut -c1-300 $OUT/slice8_tail$t.jsonl
  python3 tools/timeline.py $OUT/tl_$t > $OUT/timeline_slice8_tail$t.txt 2>&1
  cat $OUT/timeline_slice8_tail$t.txt
  rm -rf $OUT/tl_$t
done
for e in cur nbhalf3; do
  if [ -f pbrt-v2-spectral_amd/lib/exp/$e.so ]; then
    PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/$e.so timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_exp_$e.json 2> $OUT/bench_exp_$e.err || { tail -20 $OUT/bench_exp_$e.err; exit 1; }
    cut -c1-200 $OUT/bench_exp_$e.json
  fi
done
echo done
