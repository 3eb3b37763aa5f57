set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for st in 200 200 200 2000 2000; do
timeout -k 10 120 python bench.py --steps $st --no-cpu-baseline > gpurun_out/st_$st.json 2>/dev/null || exit $?
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['config']['kernel_ms'], d['config']['sync_ms_per_step'])" gpurun_out/st_$st.json $st
done
