#!/bin/bash
# r06aj: the final tree as the driver runs it -- the whole GPU suite, smoke(), the default bench line
OUT=$PWD/gpurun_out/r06aj
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/frame_parity.jsonl $OUT/ 2>/dev/null; rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_default.json'));r=d['roofline'];print('c2',d['value'],r['frac'],r['traffic'],d['setup_ms'],d['hbm_GBps'],{k:v['efficiency'] for k,v in d['slice_efficiency'].items() if k.startswith('1/')},d['cpu_baseline']['value'])"
echo done
