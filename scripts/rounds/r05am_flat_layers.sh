set -o pipefail
# r05am: wave 0 resolves the screen layers before the barrier (RT_FLAT_LAYER_EARLY)
mkdir -p gpurun_out/r05am
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py tests/test_gpu_setup.py > gpurun_out/r05am/pytest.log 2>&1 &&
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 16 --size 256 --mode flat --no-shadows --variants le0,le1=default > gpurun_out/r05am/flat.json 2> gpurun_out/r05am/flat.err &&
tail -n 2 gpurun_out/r05am/pytest.log && cat gpurun_out/r05am/flat.json
