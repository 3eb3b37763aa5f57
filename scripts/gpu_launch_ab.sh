# Frame-loop launch A/B: HIP event packets vs dispatch-packet timestamps
# (VX_HIP_EXT_LAUNCH), queue depth 1 (simx-synchronous start) .. 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-la}
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for ext in 0 1; do for qd in 1 2 4; do
  echo "== ext=$ext depth=$qd"
  VX_HIP_EXT_LAUNCH=$ext VX_HIP_QUEUE_DEPTH=$qd timeout -k 10 120 python bench.py --steps 300 --no-cpu-baseline > gpurun_out/${T}_e${ext}_q${qd}.json 2>/dev/null || exit $?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['config']['kernel_ms'], d['config']['sync_ms_per_step'], d['value'])" gpurun_out/${T}_e${ext}_q${qd}.json
done; done
