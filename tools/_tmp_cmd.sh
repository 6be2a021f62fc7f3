set -e
bash tools/gpu_cfg.sh r02d "bunny or measured or coverage" c3
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/meascheap.so timeout -k 10 200 python3 bench.py --config c3 --steps 1 --no-cpu --no-roofline > gpurun_out/r02d/cheap.json 2>gpurun_out/r02d/cheap.err
python3 -c "import json; d=json.load(open('gpurun_out/r02d/cheap.json')); print('cheap', d['value'], d['ms_per_step'])"
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/sections.so timeout -k 10 200 python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu --no-roofline > gpurun_out/r02d/sec.json 2>gpurun_out/r02d/sec.err
grep sections gpurun_out/r02d/sec.err | tail -2
