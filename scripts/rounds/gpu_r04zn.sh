# r04zn: the full GPU suite and one bench line on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-r04zn}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${T}_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json;j=json.load(open('gpurun_out/${T}_bench.json'));c=j['config'];print(j['value'],j['ms_per_step'],c['kernel_ms'],j['roofline']['frac'],{k:c[k] for k in c if 'bvh' in k})"
