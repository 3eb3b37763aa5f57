# r03w: full round on the shipped images (tests, smoke, PMC records, bench
# lines, rocprof summaries), then the 2-rank rehearsal of bench.py's N > 1
# flow on this one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03w bash scripts/gpu_round.sh || exit $?
NS=2 bash scripts/gpu_rehearsal.sh
