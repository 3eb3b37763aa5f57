# r04zc: BVH-walk form A/B -- 32-pixel waves for the geometry tiles (RT_SPLIT_TILES)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zc
echo "== bvh A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --bvh-walk --size 1024 --rounds 10 --frames 20 --variants "base=default,s16=default:RT_SPLIT_TILES=16,s64=default:RT_SPLIT_TILES=64,s256=default:RT_SPLIT_TILES=256" > gpurun_out/${T}_bvh.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bvh.log; exit $rc
