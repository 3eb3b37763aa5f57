# Grid-size sweep: VX_HIP_BLOCKS_PER_CU (64-thread blocks per CU; default
# kGridWavesPerCU) for the config 3 and config 4 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-grid}
: > gpurun_out/${T}.jsonl
for w in shadow path; do
for n in ${PER_CU:-default 16 32 48 96 128}; do
  if [ "$n" = default ]; then unset VX_HIP_BLOCKS_PER_CU; else export VX_HIP_BLOCKS_PER_CU=$n; fi
  echo "== $w per_cu $n"
  timeout -k 10 120 python bench.py --workload $w --no-cpu-baseline --steps 1000 --warmup 50 > gpurun_out/${T}_${w}_$n.json 2> gpurun_out/${T}_${w}_$n.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'workload': sys.argv[2], 'per_cu': sys.argv[3], 'grid': d['config']['grid'], 'value': d['value'], 'kernel_ms': d['config']['kernel_ms']}))" gpurun_out/${T}_${w}_$n.json $w $n | tee -a gpurun_out/${T}.jsonl
done; done
