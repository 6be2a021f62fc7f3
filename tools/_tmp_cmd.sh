set -e
mkdir -p gpurun_out/r02k
for e in base blk128 wpe4 nomis nonee; do
  if [ $e = base ]; then L=""; else L="PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/$e.so"; fi
  env $L timeout -k 10 200 python3 bench.py --config c2 --steps 2 --no-cpu > gpurun_out/r02k/$e.json 2>gpurun_out/r02k/$e.err
  python3 -c "import json; d=json.load(open('gpurun_out/r02k/$e.json')); r=d['roofline']; print('$e', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in r['kernels'].items()})"
done
