# r03k: the path tracer's cooperative lane pairs (PT_COOP) in the one-kernel
# default -- parity tests, A/B against the per-lane image, per-kernel rocprof
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03k FILES="tests/test_gpu_pt.py" \
  AB_PATH="coop=default,nocoop=nocoop,q64=default:RT_PT_QUEUE=1" \
  bash scripts/gpu_ab.sh || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03k_prof -o r03k --output-format csv -- python3 bench.py --no-cpu-baseline --workload path --steps 300 --warmup 20 > gpurun_out/r03k_bench_path.json 2> gpurun_out/r03k_bench_path.err
