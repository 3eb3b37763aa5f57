# r04c: one-workgroup climb, workgroup-per-primitive PRIMVIS, register
# projection (no scratch): setup tests, the probe under a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04c
echo "== pytest setup"; timeout -k 10 300 python -u -m pytest tests/test_gpu_light.py tests/test_gpu_setup.py tests/test_gpu_blists.py tests/test_gpu_rt.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_setup.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_setup.log; grep "cold configure" gpurun_out/${T}_pytest_setup.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_setup.log | head -20; exit $rc; }
echo "== setup probe"; RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_setup -o setup --output-format csv -- python3 scripts/setup_probe.py > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; python3 -c "
import json;d=json.load(open('gpurun_out/${T}_setup.json'))
for x in d: print(x['tag'], x.get('configure_ms'), x.get('set_light_wait_ms'), x.get('launches'))"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
