set -o pipefail
# r05ar: dense flat rounds warm the scalar cache with their candidate records (RT_FLAT_TOUCH)
mkdir -p gpurun_out/r05ar
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_flat.py > gpurun_out/r05ar/pytest.log 2>&1 &&
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 16 --size 256 --mode flat --no-shadows --variants tc0,tc1=default > gpurun_out/r05ar/flat.json 2> gpurun_out/r05ar/flat.err &&
tail -n 1 gpurun_out/r05ar/pytest.log && cat gpurun_out/r05ar/flat.json
