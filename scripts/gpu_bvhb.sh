set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== pytest bvh build"; timeout -k 10 400 python -u -m pytest tests/test_gpu_bvh_build.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/bvhb_pytest.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/bvhb_pytest.log | tail -25; [ $rc -eq 0 ] || exit $rc
echo "== bench bvh build"; timeout -k 10 400 python scripts/bench_bvh_build.py > gpurun_out/bvhb_bench.jsonl 2> gpurun_out/bvhb_bench.err; rc=$?; cat gpurun_out/bvhb_bench.jsonl; tail -3 gpurun_out/bvhb_bench.err; exit $rc
