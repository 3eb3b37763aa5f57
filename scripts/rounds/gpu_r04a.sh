# r04a: full GPU suite (layer records counted per wave, rt_bvh image, 3 list
# padding entries), the default bench line with its BVH series, the config-3
# PMC records (shadow, bvh) and the cold/warm configure probe with per-launch
# device times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04a
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_gpu.log | head -20; exit $rc; }
for m in shadow bvh; do
echo "== pmc $m"; MODE=$m TAG=${T}_pmc bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc_$m.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_$m.log; exit 1; }
cp gpurun_out/${T}_pmc/pmc_$m.json profiles/
done
echo "== bench"; timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof.log; [ $rc -eq 0 ] || exit $rc
echo "== setup probe"; RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_setup -o setup --output-format csv -- python3 scripts/setup_probe.py > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; cat gpurun_out/${T}_setup.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
