# r04n: path A/B -- the pair's stack top in a register; setup sequences as
# one untimed run (no events between steps): tests, probe, launch trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04za
echo "== pytest setup"; timeout -k 10 400 python -u -m pytest tests/test_gpu_light.py tests/test_gpu_setup.py tests/test_gpu_blists.py tests/test_gpu_rt.py tests/test_gpu_pt.py tests/test_gpu_bvh_walk.py tests/test_gpu_shard.py -x -q -s --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.log; grep "cold configure" gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
echo "== setup probe"; timeout -k 10 200 python3 scripts/setup_probe.py > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
python3 -c "
import json;d=json.load(open('gpurun_out/${T}_setup.json'))
print(' '.join('%s=%s'%(x['tag'],x.get('configure_ms',x.get('set_light_wait_ms'))) for x in d))"
echo "== setup trace"; RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/${T}_strace -o setup --output-format csv -- python3 scripts/setup_probe.py --moving 3 > gpurun_out/${T}_strace.json 2> gpurun_out/${T}_strace.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_strace.err; exit $rc; }

