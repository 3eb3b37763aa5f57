# Run-to-run spread of the default (config 3) bench line on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-repeat}
: > gpurun_out/${T}.jsonl
for i in 1 2 3 4 5; do
  echo "== run $i"
  timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/${T}_$i.json 2> gpurun_out/${T}_$i.err || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(json.dumps({'run': int(sys.argv[2]), 'value': d['value'], 'kernel_ms': d['config']['kernel_ms'], 'ms_per_step': d['ms_per_step'], 'frac': d['roofline']['frac']}))" gpurun_out/${T}_$i.json $i | tee -a gpurun_out/${T}.jsonl
done
