# The N>1 bench exchange path at world size 1 (BENCH_FORCE_GATHER): RCCL on
# one GPU checks the pipelined stream order (driver-stream copy -> torch
# stream -> gather -> assembly); gloo checks the host-staged form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-g1}
echo "== pytest gpu rt"; timeout -k 10 300 python -u -m pytest tests/test_gpu_rt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
for be in nccl gloo; do
echo "== forced gather $be"; BENCH_FORCE_GATHER=1 BENCH_DIST_BACKEND=$be timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --steps 100 --warmup 5 --verify-gather > gpurun_out/${T}_${be}.json 2> gpurun_out/${T}_${be}.err; rc=$?; cut -c1-420 gpurun_out/${T}_${be}.json; grep -h "gathered" gpurun_out/${T}_${be}.err; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_${be}.err; exit $rc; }
done
