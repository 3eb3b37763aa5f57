# Frame assembly kernel: GPU tests, microbench vs index_select, forced-gather
# bench (RCCL at world size 1) with frame verification at two sizes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-asm}
echo "== pytest"; timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_rt.py tests/test_gpu_pt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== microbench"; timeout -k 10 200 python scripts/bench_assemble.py > gpurun_out/${T}_micro.jsonl 2> gpurun_out/${T}_micro.err; rc=$?; cat gpurun_out/${T}_micro.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_micro.err; exit $rc; }
for sz in 1024 2896; do
echo "== forced gather nccl $sz"; BENCH_FORCE_GATHER=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --size $sz --steps 200 --warmup 10 --no-cpu-baseline --verify-gather > gpurun_out/${T}_g$sz.json 2> gpurun_out/${T}_g$sz.err; rc=$?; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['config'].get('kernel_ms'), d['value'])" gpurun_out/${T}_g$sz.json; grep -h "gathered" gpurun_out/${T}_g$sz.err; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_g$sz.err; exit $rc; }
echo "== plain $sz"; timeout -k 10 200 python bench.py --size $sz --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/${T}_p$sz.json 2> gpurun_out/${T}_p$sz.err; rc=$?; python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['config'].get('kernel_ms'), d['value'])" gpurun_out/${T}_p$sz.json; [ $rc -eq 0 ] || exit $rc
done
