# Multi-rank rehearsal of bench.py's N>1 flow on ONE GPU: `--gpus N` launches
# N ranks itself, all on cuda:0, exchanging through host-staged gloo gathers
# (RCCL refuses two ranks on one device); config 5's 4096^2 tile-sharded
# frame, the gathered + assembled frame verified against a full render.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for n in ${NS:-2 8}; do
echo "== ranks $n"
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n --steps ${STEPS:-20} --warmup 3 --verify-gather --no-cpu-baseline --no-series > gpurun_out/rehearsal_${n}rank.json 2> gpurun_out/rehearsal_${n}rank.err || { tail -20 gpurun_out/rehearsal_${n}rank.err; exit 1; }
cat gpurun_out/rehearsal_${n}rank.json
done
