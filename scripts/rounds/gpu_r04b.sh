# r04b: the stream-ordered setup sequence and the moving light -- the setup
# and list tests first, then the whole suite, the bench line (with its
# bvh_walk and moving_light series) and the setup probe under a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04b
echo "== pytest setup"; timeout -k 10 300 python -u -m pytest tests/test_gpu_light.py tests/test_gpu_setup.py tests/test_gpu_blists.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_setup.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_setup.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_setup.log | head -20; exit $rc; }
grep "cold configure" gpurun_out/${T}_pytest_setup.log
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_gpu.log | head -20; exit $rc; }
echo "== bench"; timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err; rc=$?; cat gpurun_out/${T}_bench.json; tail -2 gpurun_out/${T}_bench.err; [ $rc -eq 0 ] || exit $rc
echo "== setup probe"; RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_setup -o setup --output-format csv -- python3 scripts/setup_probe.py > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; cat gpurun_out/${T}_setup.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
echo "== ab xcd"; timeout -k 10 250 python scripts/ab_variants.py --rounds 10 --variants "default,xcd" > gpurun_out/${T}_ab_xcd.json 2> gpurun_out/${T}_ab_xcd.err; rc=$?; cat gpurun_out/${T}_ab_xcd.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_ab_xcd.err; exit $rc; }
echo "== ab flat"; timeout -k 10 250 python scripts/ab_variants.py --mode flat --size 256 --no-shadows --rounds 10 --variants "default,flat512,flat1024" > gpurun_out/${T}_ab_flat.json 2> gpurun_out/${T}_ab_flat.err; rc=$?; cat gpurun_out/${T}_ab_flat.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_ab_flat.err; exit $rc; }
