# One GPU call: pytest -m gpu, smoke, PMC traffic passes, bench (with CPU
# baseline), rocprof kernel-trace summary of the same bench command, A/B.
# TAG names the outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-run}
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
for m in shadow path flat; do
echo "== traffic $m"; MODE=$m TAG=${T}_traffic bash scripts/pmc_traffic.sh || exit $?
done
cp gpurun_out/${T}_traffic/pmc_traffic*.json profiles/
echo "== bench"; timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
echo "== bench path"; timeout -k 10 300 python bench.py --workload path --cpu-budget 5 > gpurun_out/${T}_bench_path.json 2> gpurun_out/${T}_bench_path.err; rc=$?; cat gpurun_out/${T}_bench_path.json; tail -2 gpurun_out/${T}_bench_path.err; [ $rc -eq 0 ] || exit $rc
echo "== bench flat"; timeout -k 10 300 python bench.py --workload flat --cpu-budget 5 > gpurun_out/${T}_bench_flat.json 2> gpurun_out/${T}_bench_flat.err; rc=$?; cat gpurun_out/${T}_bench_flat.json; tail -2 gpurun_out/${T}_bench_flat.err; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$AB" ]; then echo "== ab"; timeout -k 10 250 python scripts/ab_variants.py --rounds 8 --variants "$AB" > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err; rc=$?; cat gpurun_out/${T}_ab.json; exit $rc; fi
