# r04z: round-end evidence on the shipped images -- full GPU suite, PMC
# records of the four timed images (shadow, bvh, path, flat), the bench lines
# (config 3 with its BVH / moving-light series and cold configure; config 4;
# config 2) and their rocprofv3 kernel-trace summaries, the setup probe, and
# the roofline check over them
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-r04z2}
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; grep "cold configure" gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_gpu.log | head -20; exit $rc; }
for m in shadow bvh path flat; do
  echo "== pmc $m"; MODE=$m TAG=${T}_pmc bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc_$m.log 2>&1 || { tail -5 gpurun_out/${T}_pmc_$m.log; exit 1; }
  cp gpurun_out/${T}_pmc/pmc_$m.json profiles/
done
for w in shadow path flat; do
  echo "== bench $w"; timeout -k 10 400 python bench.py --workload $w > gpurun_out/${T}_bench_$w.json 2> gpurun_out/${T}_bench_$w.err; rc=$?; head -c 600 gpurun_out/${T}_bench_$w.json; echo; tail -2 gpurun_out/${T}_bench_$w.err; [ $rc -eq 0 ] || exit $rc
  echo "== rocprof $w"; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$w -o ${T}_$w --output-format csv -- python3 bench.py --workload $w --no-cpu-baseline > gpurun_out/${T}_prof_$w.json 2> gpurun_out/${T}_prof_$w.err; rc=$?; [ $rc -eq 0 ] || { tail -3 gpurun_out/${T}_prof_$w.err; exit $rc; }
done
echo "== setup probe"; timeout -k 10 200 python3 scripts/setup_probe.py > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
echo done
