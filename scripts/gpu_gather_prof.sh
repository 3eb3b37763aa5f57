# Timeline of the pipelined exchange at world size 1 (RCCL to self):
# kernel + memory-copy trace of bench.py's forced-gather path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-gp}
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29543 BENCH_FORCE_GATHER=1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_prof.log | cut -c1-300; exit $rc
