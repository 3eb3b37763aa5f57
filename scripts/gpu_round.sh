# One GPU call: pytest -m gpu, smoke, the PMC record of every bench workload
# (scripts/pmc_profile.sh -> profiles/pmc_<mode>.json), the bench lines
# (config 3 with the CPU baseline, config 4, config 2) and the rocprofv3
# kernel-trace summary of the default bench command.  TAG names the outputs
# under gpurun_out/; every GPU step has its own time limit and the first
# failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-run}
step() { echo "== $1"; }
if [ -z "$NO_TESTS" ]; then
step "pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
step "smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NO_PMC" ]; then
for m in shadow path flat; do
step "pmc $m"; MODE=$m TAG=${T}_pmc bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc_$m.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_$m.log; exit 1; }
cp gpurun_out/${T}_pmc/pmc_$m.json profiles/
done
fi
step "bench"; timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
step "bench path"; timeout -k 10 300 python bench.py --workload path --cpu-budget 5 > gpurun_out/${T}_bench_path.json 2> gpurun_out/${T}_bench_path.err; rc=$?; cat gpurun_out/${T}_bench_path.json; tail -2 gpurun_out/${T}_bench_path.err; [ $rc -eq 0 ] || exit $rc
step "bench flat"; timeout -k 10 300 python bench.py --workload flat --cpu-budget 5 > gpurun_out/${T}_bench_flat.json 2> gpurun_out/${T}_bench_flat.err; rc=$?; cat gpurun_out/${T}_bench_flat.json; tail -2 gpurun_out/${T}_bench_flat.err; [ $rc -eq 0 ] || exit $rc
step "rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof.log; [ $rc -eq 0 ] || exit $rc
step "rocprof path"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_path -o ${T}_path --output-format csv -- python3 bench.py --no-cpu-baseline --workload path > gpurun_out/${T}_prof_path.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof_path.log; [ $rc -eq 0 ] || exit $rc
step "rocprof flat"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_flat -o ${T}_flat --output-format csv -- python3 bench.py --no-cpu-baseline --workload flat > gpurun_out/${T}_prof_flat.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof_flat.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$AB" ]; then step "ab"; timeout -k 10 250 python scripts/ab_variants.py --rounds 8 --variants "$AB" > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err; rc=$?; cat gpurun_out/${T}_ab.json; exit $rc; fi
