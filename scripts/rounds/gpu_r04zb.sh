# r04zb: BVH-walk form A/B -- workgroup size
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zb
echo "== bvh A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --bvh-walk --size 1024 --rounds 10 --frames 20 --variants "b256=default,xcd=bvhxcd" > gpurun_out/${T}_bvh.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_bvh.log; exit $rc
