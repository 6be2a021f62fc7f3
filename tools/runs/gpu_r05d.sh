#!/bin/bash
# r05d: the quantized 4-wide shadow BVH (k_trace_s4q) -- GPU suite (intersect KAT with all three
# shadow walks, goldens, full frames), then A/B against the exact 4-wide walk (PBRTGPU_SHADOW4Q=0)
# on C2 and C2 DirectLighting (two rounds), L2 hit rates of the shadow kernel both ways; the slot
# pool of a 1/8 slice (spatial locality of a generation vs fill / drain); C3 / C4 / C5 bench lines
OUT=$PWD/gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -30 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for x in 1 0; do
    PBRTGPU_SHADOW4Q=$x timeout -k 10 300 python3 bench.py --no-cpu > $OUT/bench_c2_q${x}_$r.json 2> $OUT/bench_c2_q${x}_$r.err || { tail -20 $OUT/bench_c2_q${x}_$r.err; exit 1; }
    cut -c1-200 $OUT/bench_c2_q${x}_$r.json
    PBRTGPU_SHADOW4Q=$x timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl_q${x}_$r.json 2> $OUT/bench_dl_q${x}_$r.err || { tail -20 $OUT/bench_dl_q${x}_$r.err; exit 1; }
    cut -c1-200 $OUT/bench_dl_q${x}_$r.json
  done
done
for x in 1 0; do
  PBRTGPU_SHADOW4Q=$x timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc_$x -o run -- python3 bench.py --no-cpu --no-roofline --no-slices --steps 1 --warmup 0 --serial > $OUT/pmc_tcc_$x.json 2> $OUT/pmc_tcc_$x.err || { tail -20 $OUT/pmc_tcc_$x.err; exit 1; }
  python3 tools/pmc_table.py $OUT/pmc_tcc_$x > $OUT/pmc_tcc_$x.txt 2>&1
  PBRTGPU_SHADOW4Q=$x timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc_dl_$x -o run -- python3 bench.py --integrator directlighting --no-cpu --no-roofline --no-slices --steps 1 --warmup 0 --serial > $OUT/pmc_tcc_dl_$x.json 2> $OUT/pmc_tcc_dl_$x.err || { tail -20 $OUT/pmc_tcc_dl_$x.err; exit 1; }
  python3 tools/pmc_table.py $OUT/pmc_tcc_dl_$x > $OUT/pmc_tcc_dl_$x.txt 2>&1
  rm -rf $OUT/pmc_tcc_$x $OUT/pmc_tcc_dl_$x
done
for s in 2097152 4194304 8388608; do
  PBRTGPU_SLOTS=$s timeout -k 10 200 python3 tools/slice_run.py --slice 8 --reps 3 > $OUT/slice8_slots$s.jsonl 2> $OUT/slice8_slots$s.err || { tail -20 $OUT/slice8_slots$s.err; exit 1; }
  cut -c1-260 $OUT/slice8_slots$s.jsonl
done
for c in c3 c4 c5; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-slices > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -20 $OUT/bench_$c.err; exit 1; }
  cut -c1-200 $OUT/bench_$c.json
done
echo done
