# Quick GPU check: pytest -m gpu, then the three bench lines without the CPU
# baseline.  TAG names the outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-quick}
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_gpu.log | head -20; exit $rc; }
for w in shadow path flat; do
echo "== bench $w"; timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/${T}_bench_$w.json 2> gpurun_out/${T}_bench_$w.err; rc=$?; python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench_$w.json'));print(d['value'],d['ms_per_step'],d['config']['kernel_ms'],d['roofline']['counts'])"; [ $rc -eq 0 ] || exit $rc
done
