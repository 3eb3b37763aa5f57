set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-g2}
echo "== forced gather nccl"; BENCH_FORCE_GATHER=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --steps 200 --warmup 5 --verify-gather > gpurun_out/${T}_nccl.json 2> gpurun_out/${T}_nccl.err; rc=$?; cut -c1-400 gpurun_out/${T}_nccl.json; grep -h "gathered" gpurun_out/${T}_nccl.err; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_nccl.err; exit $rc; }
echo "== rehearse 2 ranks (gloo)"; BENCH_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --verify-gather > gpurun_out/${T}_rehearse2.json 2> gpurun_out/${T}_rehearse2.err; rc=$?; cut -c1-300 gpurun_out/${T}_rehearse2.json; grep -h "gathered" gpurun_out/${T}_rehearse2.err; [ $rc -eq 0 ] || exit $rc
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29543 BENCH_FORCE_GATHER=1
echo "== prof"; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o ${T} --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_prof.log | cut -c1-200; exit $rc
