# path tracer parity tests + A/B of path-tracer image variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-pt}
echo "== pytest gpu pt"; timeout -k 10 300 python -u -m pytest tests/test_gpu_pt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== ab path"; timeout -k 10 250 python scripts/ab_variants.py --mode path --rounds 8 --variants "$AB" > gpurun_out/${T}_ab_path.json 2> gpurun_out/${T}_ab_path.err; rc=$?; cat gpurun_out/${T}_ab_path.json; tail -2 gpurun_out/${T}_ab_path.err; exit $rc
