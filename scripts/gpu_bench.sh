# bench lines (config 3 with CPU baseline, config 4) + rocprof kernel-trace
# summary of the default bench command.  TAG names the outputs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-bench}
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/${T}_bench.err; exit $rc; }
echo "== bench path"; timeout -k 10 300 python bench.py --workload path --cpu-budget 5 > gpurun_out/${T}_bench_path.json 2> gpurun_out/${T}_bench_path.err; rc=$?; cat gpurun_out/${T}_bench_path.json; [ $rc -eq 0 ] || exit $rc
echo "== bench flat"; timeout -k 10 300 python bench.py --workload flat --cpu-budget 5 > gpurun_out/${T}_bench_flat.json 2> gpurun_out/${T}_bench_flat.err; rc=$?; cat gpurun_out/${T}_bench_flat.json; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof.log; exit $rc
