#!/bin/bash
# r06am: the rebuilt final libraries (same source) -- the whole GPU suite and smoke()
OUT=$PWD/gpurun_out/r06am
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -2 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/frame_parity.jsonl
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo done
