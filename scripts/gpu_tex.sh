# tex app: GPU tests, throughput, rocprof kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-tex}
echo "== pytest tex"; timeout -k 10 300 python -u -m pytest tests/test_gpu_tex.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== bench tex"; timeout -k 10 300 python scripts/bench_tex.py > gpurun_out/${T}_bench.jsonl 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.jsonl; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
echo "== rocprof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 scripts/bench_tex.py --steps 20 --cpu-budget 0.1 > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof.log; exit $rc
