# A/B: while-while traversal loop (RT_WW) vs if-if, shadow and path modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-ww}
echo "== pytest gpu rt/pt"; timeout -k 10 300 python -u -m pytest tests/test_gpu_rt.py tests/test_gpu_pt.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== ab shadow"; timeout -k 10 200 python scripts/ab_variants.py --rounds 10 --variants "${ABS:-base=default,ww}" > gpurun_out/${T}_shadow.json 2> gpurun_out/${T}_shadow.err; rc=$?; cat gpurun_out/${T}_shadow.json; grep -c "identical=False" gpurun_out/${T}_shadow.err; [ $rc -eq 0 ] || exit $rc
echo "== ab path"; timeout -k 10 200 python scripts/ab_variants.py --mode path --rounds 10 --variants "${ABP:-base=default,ptww}" > gpurun_out/${T}_path.json 2> gpurun_out/${T}_path.err; rc=$?; cat gpurun_out/${T}_path.json; grep -c "identical=False" gpurun_out/${T}_path.err; exit $rc
