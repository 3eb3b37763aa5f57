# r04i: path tracer node step with one exchange round (local sort): parity + A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04i
echo "== pytest pt"; timeout -k 10 400 python -u -m pytest tests/test_gpu_pt.py tests/test_gpu_light.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
echo "== path A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 8 --frames 10 --variants "local=default,net3=coop0" > gpurun_out/${T}_path.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_path.log; [ $rc -eq 0 ] || exit $rc
echo "== flat grid"; timeout -k 10 200 python3 scripts/ab_variants.py --mode flat --no-shadows --size 256 --rounds 10 --frames 20 --variants "g16=default,g4=default:VX_HIP_BLOCKS_PER_CU=4,g8=default:VX_HIP_BLOCKS_PER_CU=8" > gpurun_out/${T}_flat.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_flat.log; exit $rc
