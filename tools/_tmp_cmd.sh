set -e
bash tools/gpu_cfg.sh r02i "anim or instance or inst" c5
PBRTGPU_LIB=$PWD/pbrt-v2-spectral_amd/lib/exp/inst3.so timeout -k 10 200 python3 bench.py --config c5 --steps 1 --no-cpu > gpurun_out/r02i/i3.json 2>gpurun_out/r02i/i3.err
python3 -c "import json; d=json.load(open('gpurun_out/r02i/i3.json')); r=d['roofline']; print('inst3', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in r['kernels'].items()})"
PBRTGPU_INST_WALK=legacy timeout -k 10 200 python3 bench.py --config c5 --steps 1 --no-cpu > gpurun_out/r02i/leg.json 2>gpurun_out/r02i/leg.err
python3 -c "import json; d=json.load(open('gpurun_out/r02i/leg.json')); r=d['roofline']; print('legacy', d['value'], d['ms_per_step'], {k: v['ms_per_frame'] for k, v in r['kernels'].items()})"
