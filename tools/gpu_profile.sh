#!/bin/bash
# GPU-box profiling recipe for one config: rocprofv3 kernel trace + stats of the bench
# command (default mode and serial mode), then separate PMC passes (FETCH_SIZE, WRITE_SIZE,
# two SQ groups) over one serial-mode frame (no concurrent kernels: one frame's launches,
# each counted once).  Usage (repo root, GPU box): bash tools/gpu_profile.sh TAG [config [bench args]]
# (e.g. bash tools/gpu_profile.sh r02n_dl c2 --integrator directlighting)
set -e
TAG=${1:-r02}
CFG=${2:-c2}
shift 2 || true
EXTRA="$*"
OUT=$PWD/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --config $CFG --no-cpu --no-roofline --no-slices $EXTRA"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 $B --steps 2 --warmup 1 > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_serial -o run -- python3 $B --steps 1 --warmup 1 --serial > $OUT/bench_trace_serial.json 2> $OUT/trace_serial.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/pmc1.json 2> $OUT/pmc1.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/pmc2.json 2> $OUT/pmc2.err
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $OUT/pmc_sq1 -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/pmc3.json 2> $OUT/pmc3.err
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_sq2 -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/pmc4.json 2> $OUT/pmc4.err
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $OUT/pmc_lds -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/pmc5.json 2> $OUT/pmc5.err || echo "LDS pass failed (counter set not available)"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc -o run -- python3 $B --steps 1 --warmup 0 --serial > $OUT/pmc6.json 2> $OUT/pmc6.err || echo "TCC pass failed"
# summaries next to the run (gpurun_out is copied back only below 64 MiB): the rocpd databases go
SUMCFG=$CFG; case "$EXTRA" in *directlighting*) SUMCFG=${CFG}_dl;; *metadata*) SUMCFG=${CFG}_meta;; esac
case "$EXTRA" in *spectral*) SUMCFG=${SUMCFG}_spec;; esac
python3 tools/rocpd_summary.py $TAG $OUT $SUMCFG $PWD/gpurun_out/summaries > /dev/null
rm -rf $OUT/trace $OUT/trace_serial $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_sq1 $OUT/pmc_sq2 $OUT/pmc_lds $OUT/pmc_tcc
echo done
