#!/bin/bash
# r05m: C3 on the measured-BRDF-only k_shade / k_tail build (FEAT_MEAS, 32 bands) against the
# all-features build (PBRTGPU_SHADE_FULL=1), after the loop-free kd radius; the BxDF kind chosen
# once per band quad (C2, DirectLighting); parity first (the whole GPU suite)
OUT=$PWD/gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
for m in 0 1 0 1; do
PBRTGPU_SHADE_FULL=$m timeout -k 10 300 python3 bench.py --config c3 --no-cpu --no-slices > $OUT/bench_c3_f$m.json 2> $OUT/bench_c3_f$m.err || { tail -20 $OUT/bench_c3_f$m.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c3_f$m.json'));k=d['roofline']['kernels'];print('full$m',d['value'],k['k_shade']['ms_per_frame'])"
done
echo done
for i in 1 2; do
timeout -k 10 300 python3 bench.py --no-cpu --no-slices > $OUT/bench_c2_$i.json 2> $OUT/bench_c2_$i.err || { tail -20 $OUT/bench_c2_$i.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c2_$i.json'));k=d['roofline']['kernels'];print('c2',d['value'],k['k_shade']['ms_per_frame'])"
done
timeout -k 10 300 python3 bench.py --integrator directlighting --no-cpu --no-slices > $OUT/bench_dl.json 2> $OUT/bench_dl.err || { tail -20 $OUT/bench_dl.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_dl.json'));k=d['roofline']['kernels'];print('dl',d['value'],k['k_shade']['ms_per_frame'])"
# PC sampling (host trap) of one C2 frame: where k_shade's issue slots go
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 4 -d $OUT/pcs -o pcs --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-slices --no-roofline > $OUT/pcs.log 2>&1
echo "pcs rc $?"
tail -5 $OUT/pcs.log
find $OUT/pcs -type f
ls -la $OUT/pcs/*/ 2>/dev/null || true
