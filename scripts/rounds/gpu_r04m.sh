# r04m: leaf interleave default: path parity; 16-pixel pair waves for the heaviest tiles (RT_QUAD_TILES, pairs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04m
echo "== pytest pt"; timeout -k 10 400 python -u -m pytest tests/test_gpu_pt.py tests/test_gpu_light.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
echo "== path A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 8 --frames 10 --variants "base=default,topreg=topreg,q8=default:RT_QUAD_TILES=8,q16=default:RT_QUAD_TILES=16,q32=default:RT_QUAD_TILES=32" > gpurun_out/${T}_path.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_path.log; exit $rc
