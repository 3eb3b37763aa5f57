set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r4_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r4_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== ab"; timeout -k 10 300 python scripts/ab_variants.py --rounds 8 > gpurun_out/r4_ab.json 2> gpurun_out/r4_ab.err; rc=$?; cat gpurun_out/r4_ab.json; grep identical gpurun_out/r4_ab.err | cut -c1-40; exit $rc
