# r03o: the kernel clock (HIP events around back-to-back untimed frames)
# against rocprofv3's per-dispatch average in the same command
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_rt.py -x -q -k queued --timeout 120 --timeout-method thread > gpurun_out/r03o_pytest.log 2>&1 || { tail -20 gpurun_out/r03o_pytest.log; exit 1; }
tail -1 gpurun_out/r03o_pytest.log
for w in shadow flat path; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03o_prof_$w -o r03o_$w --output-format csv -- python3 bench.py --no-cpu-baseline --workload $w > gpurun_out/r03o_bench_$w.json 2> gpurun_out/r03o_bench_$w.err || exit 1
done
