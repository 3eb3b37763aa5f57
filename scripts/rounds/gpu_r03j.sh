# r03j: segmented path queue + the one-loop vertex (PT_ILP) -- parity tests,
# A/B of the four path-tracer forms, per-kernel rocprof summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03j FILES="tests/test_gpu_pt.py" \
  AB_PATH="q64=default,one=default:RT_PT_QUEUE=0,ilpq=ilp,ilp1=ilp:RT_PT_QUEUE=0" \
  bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03j_prof -o r03j --output-format csv -- python3 bench.py --no-cpu-baseline --workload path --steps 300 --warmup 20 > gpurun_out/r03j_bench_path.json 2> gpurun_out/r03j_bench_path.err
