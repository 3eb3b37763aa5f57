# pytest -m gpu, pipelined bench (config 3 + 4), A/B of kernel variants in
# shadow and path modes, 2-rank gloo rehearsal of the N>1 bench path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r6}
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 300 python bench.py --cpu-budget 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
echo "== bench path"; timeout -k 10 300 python bench.py --workload path --no-cpu-baseline > gpurun_out/${T}_bench_path.json 2> gpurun_out/${T}_bench_path.err; rc=$?; cat gpurun_out/${T}_bench_path.json; [ $rc -eq 0 ] || exit $rc
if [ -n "$AB" ]; then
echo "== ab shadow"; timeout -k 10 250 python scripts/ab_variants.py --rounds 8 --variants "$AB" > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err; rc=$?; cat gpurun_out/${T}_ab.json; [ $rc -eq 0 ] || exit $rc
echo "== ab path"; timeout -k 10 250 python scripts/ab_variants.py --mode path --rounds 6 --variants "$AB" > gpurun_out/${T}_ab_path.json 2> gpurun_out/${T}_ab_path.err; rc=$?; cat gpurun_out/${T}_ab_path.json; [ $rc -eq 0 ] || exit $rc
fi
echo "== rehearse 2 ranks (gloo)"; BENCH_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --verify-gather > gpurun_out/${T}_rehearse2.json 2> gpurun_out/${T}_rehearse2.err; rc=$?; cat gpurun_out/${T}_rehearse2.json; grep -h "gathered" gpurun_out/${T}_rehearse2.err; exit $rc
