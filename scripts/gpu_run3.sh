set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r3_pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/r3_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== ab"; timeout -k 10 300 python scripts/ab_variants.py > gpurun_out/r3_ab.json 2> gpurun_out/r3_ab.err; rc=$?; cat gpurun_out/r3_ab.json; tail -4 gpurun_out/r3_ab.err; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-budget 3 > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err; rc=$?; cat gpurun_out/r3_bench.json; exit $rc
