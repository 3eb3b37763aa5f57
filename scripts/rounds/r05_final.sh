set -o pipefail
STEPS="tests bench smoke" TAG=r05au WORKLOADS="shadow path flat" bash scripts/rounds/gpu_r05.sh || exit 1
for i in 1 2 3; do timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05au_drv$i.json 2> gpurun_out/r05au_drv$i.err || exit 1; python3 -c "import json;j=json.load(open('gpurun_out/r05au_drv$i.json'));c=j['config'];print('drv',$i,j['value'],j['ms_per_step'],c['kernel_ms'],c['sync_ms_per_step'])"; done
STEPS="prof" TAG=r05au WORKLOADS="shadow path flat" bash scripts/rounds/gpu_r05.sh || exit 1
