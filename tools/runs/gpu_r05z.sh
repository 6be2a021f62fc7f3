#!/bin/bash
# r05z: GPU suite after the noise textures, smoke, C4 line
# metal line (textures go through tex_map now)
OUT=$PWD/gpurun_out/r05z
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -8 $OUT/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python3 bench.py --config c4 --no-cpu --no-slices > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -20 $OUT/bench_c4.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/bench_c4.json'));print('c4',d['value'],{n:v['ms_per_frame'] for n,v in d['roofline']['kernels'].items()})"
echo done
