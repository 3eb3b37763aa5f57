set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${TAG:-gap}
echo "== pytest gpu rt"; timeout -k 10 300 python -u -m pytest tests/test_gpu_rt.py tests/test_gpu_pt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for te in 1 4 8; do for mode in shadow path; do
  VX_HIP_TIME_EVERY=$te timeout -k 10 120 python scripts/launch_gap.py $mode >> gpurun_out/${T}.jsonl 2>/dev/null || exit $?
done; done
VX_HIP_EXT_LAUNCH=2 timeout -k 10 120 python scripts/launch_gap.py shadow >> gpurun_out/${T}.jsonl 2>/dev/null || exit $?
cat gpurun_out/${T}.jsonl
echo "== bench"; timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cut -c1-900 gpurun_out/${T}_bench.json; exit $rc
