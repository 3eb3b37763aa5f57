set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5}
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== ab"; timeout -k 10 300 python scripts/ab_variants.py --rounds 6 ${AB_VARIANTS:+--variants $AB_VARIANTS} > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err; rc=$?; cat gpurun_out/${T}_ab.json; grep identical gpurun_out/${T}_ab.err | cut -c1-40; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-budget 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_prof.log; exit $rc
