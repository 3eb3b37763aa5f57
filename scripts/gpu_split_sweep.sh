# Config 4 sweep of RT_SPLIT_TILES (how many of the heaviest 32x32 tiles run
# 32 pixels per wave; default = every tile geometry touches).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-split}
: > gpurun_out/${T}.jsonl
for n in ${SPLITS:-default 0 64 128 256 384 512 768 1024}; do
  if [ "$n" = default ]; then unset RT_SPLIT_TILES; else export RT_SPLIT_TILES=$n; fi
  echo "== split $n"
  timeout -k 10 120 python bench.py --workload path --no-cpu-baseline --steps 1000 --warmup 50 > gpurun_out/${T}_$n.json 2> gpurun_out/${T}_$n.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'split': sys.argv[2], 'value': d['value'], 'kernel_ms': d['config']['kernel_ms'], 'ms_per_step': d['ms_per_step']}))" gpurun_out/${T}_$n.json $n | tee -a gpurun_out/${T}.jsonl
done
