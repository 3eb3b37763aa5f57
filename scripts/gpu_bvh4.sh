set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== pytest"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/b4_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/b4_pytest.log; [ $rc -eq 0 ] || exit $rc
echo "== ab shadow"; timeout -k 10 200 python scripts/ab_variants.py --rounds 8 --variants "bvh4=default,bvh2=default:RT_BVH_WIDTH=2" > gpurun_out/b4_ab.json 2> gpurun_out/b4_ab.err; rc=$?; cat gpurun_out/b4_ab.json; [ $rc -eq 0 ] || exit $rc
echo "== ab path"; timeout -k 10 200 python scripts/ab_variants.py --mode path --rounds 8 --variants "bvh4=default,bvh2=default:RT_BVH_WIDTH=2" > gpurun_out/b4_ab_path.json 2> gpurun_out/b4_ab_path.err; rc=$?; cat gpurun_out/b4_ab_path.json; [ $rc -eq 0 ] || exit $rc
echo "== ab primary 4096"; timeout -k 10 200 python scripts/ab_variants.py --size 4096 --rounds 4 --variants "bvh4=default,bvh2=default:RT_BVH_WIDTH=2" > gpurun_out/b4_ab_4k.json 2> gpurun_out/b4_ab_4k.err; rc=$?; cat gpurun_out/b4_ab_4k.json; exit $rc
