#!/bin/bash
# r05a: round-5 baseline of the round-4 tree -- the box's CPU share (cgroup quota), the
# driver's default bench line (C2 with slices and CPU leg), C2 DirectLighting (light-sample
# list, never measured), the 1/8 slice pass log (serial and overlapped), then the C2 and
# C2 DirectLighting profiles (rocprof trace + PMC, tools/gpu_profile.sh)
OUT=$PWD/gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "OMP", os.environ.get("OMP_NUM_THREADS"))'; } > $OUT/cpu_share.txt 2>&1
cat $OUT/cpu_share.txt
timeout -k 10 400 python3 bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
cut -c1-600 $OUT/bench_c2.json
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_c2_dl.json 2> $OUT/bench_c2_dl.err || { tail -20 $OUT/bench_c2_dl.err; exit 1; }
cut -c1-600 $OUT/bench_c2_dl.json
PBRTGPU_PASS_LOG=1 timeout -k 10 200 python3 tools/slice_run.py --slice 8 --reps 2 > $OUT/slice8.jsonl 2> $OUT/slice8.passlog || { tail -20 $OUT/slice8.passlog; exit 1; }
PBRTGPU_PASS_LOG=1 PBRTGPU_SERIAL=1 timeout -k 10 200 python3 tools/slice_run.py --slice 8 --reps 1 > $OUT/slice8_serial.jsonl 2> $OUT/slice8_serial.passlog || { tail -20 $OUT/slice8_serial.passlog; exit 1; }
PBRTGPU_PASS_LOG=1 PBRTGPU_SERIAL=1 timeout -k 10 200 python3 tools/slice_run.py --slice 1 --reps 1 > $OUT/full_serial.jsonl 2> $OUT/full_serial.passlog || { tail -20 $OUT/full_serial.passlog; exit 1; }
cut -c1-400 $OUT/slice8.jsonl $OUT/slice8_serial.jsonl $OUT/full_serial.jsonl
bash tools/gpu_profile.sh r05a_dl c2 --integrator directlighting && bash tools/gpu_profile.sh r05a c2
