# Round-end evidence (r06): GPU tests + smoke, the driver's own command three
# times (profiles/r06/final/drv<i>.json), then the rocprofv3 kernel trace +
# stats of that command (profiles/r06/prof/).  TAG names the outputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r06i}
STEPS="${PRE_STEPS:-tests smoke}" TAG=$T bash scripts/rounds/gpu_r05.sh || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_drv$i.json 2> gpurun_out/${T}_drv$i.err || { tail -5 gpurun_out/${T}_drv$i.err; exit 1; }
  python3 -c "import json;j=json.load(open('gpurun_out/${T}_drv$i.json'));c=j['config'];s=j['series'];print('drv',$i,j['value'],j['ms_per_step'],c['kernel_ms'],j['roofline']['frac'],*[(k,v.get('kernel_ms'),(v.get('roofline') or {}).get('frac')) for k,v in s.items()])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv \
  -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.err \
  || { tail -5 gpurun_out/${T}_prof.err; exit 1; }
echo prof ok
