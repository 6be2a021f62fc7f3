#!/bin/bash
# r04l: the slot-pool performance mode of C2's 1/4 slice: the slice at the
# default pool (8.39 M slots per lane) and at exactly half its items (7.84 M, the slow mode of
# round 3), timed, then in serial mode with TCC hit / miss, DRAM read requests and fetch size;
# then the DirectLighting profile of the light-sample list build (tools/gpu_profile.sh)
OUT=$PWD/gpurun_out/r04l
mkdir -p $OUT
export TMPDIR=/tmp
for S in 16777216 15681600; do
  PBRTGPU_SLOTS=$S timeout -k 10 200 python3 tools/slice_run.py --slice 4 --reps 3 > $OUT/slice4_$S.jsonl 2> $OUT/slice4_$S.err || { tail -20 $OUT/slice4_$S.err; exit 1; }
  cat $OUT/slice4_$S.jsonl | cut -c1-400
  PBRTGPU_SLOTS=$S PBRTGPU_SERIAL=1 PBRTGPU_PASS_LOG=1 timeout -k 10 200 python3 tools/slice_run.py --slice 4 --reps 1 > $OUT/slice4_serial_$S.jsonl 2> $OUT/slice4_serial_$S.passlog || { tail -20 $OUT/slice4_serial_$S.passlog; exit 1; }
  cat $OUT/slice4_serial_$S.jsonl | cut -c1-400
  PBRTGPU_SLOTS=$S PBRTGPU_SERIAL=1 timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -d $OUT/pmc_tcc_$S -o run -- python3 tools/slice_run.py --slice 4 --reps 1 > $OUT/pmc_tcc_$S.jsonl 2> $OUT/pmc_tcc_$S.err || { tail -20 $OUT/pmc_tcc_$S.err; exit 1; }
  PBRTGPU_SLOTS=$S PBRTGPU_SERIAL=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$S -o run -- python3 tools/slice_run.py --slice 4 --reps 1 > $OUT/pmc_fetch_$S.jsonl 2> $OUT/pmc_fetch_$S.err || { tail -20 $OUT/pmc_fetch_$S.err; exit 1; }
  PBRTGPU_SLOTS=$S PBRTGPU_SERIAL=1 timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/pmc_sq_$S -o run -- python3 tools/slice_run.py --slice 4 --reps 1 > $OUT/pmc_sq_$S.jsonl 2> $OUT/pmc_sq_$S.err || { tail -20 $OUT/pmc_sq_$S.err; exit 1; }
done
for S in 16777216 15681600; do
  echo "== PBRTGPU_SLOTS=$S" >> $OUT/pmc_summary.txt
  python3 tools/pmc_table.py $OUT/pmc_tcc_$S $OUT/pmc_fetch_$S $OUT/pmc_sq_$S >> $OUT/pmc_summary.txt 2>&1
done
rm -rf $OUT/pmc_tcc_*/ $OUT/pmc_fetch_*/ $OUT/pmc_sq_*/
bash tools/gpu_profile.sh r04l_dl c2 --integrator directlighting
