set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r2_smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r2_pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/r2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/r2_bench.json 2> gpurun_out/r2_bench.err; rc=$?; cat gpurun_out/r2_bench.json; tail -3 gpurun_out/r2_bench.err; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r2_prof.log 2>&1; rc=$?; tail -3 gpurun_out/r2_prof.log; find gpurun_out/prof_r2 -name "*stats*"; exit $rc
