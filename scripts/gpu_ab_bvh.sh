# A/B of BVH build knobs (leaf size, SAH bins, SAH axes) and widths, shadow + path modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V="base=default,bvh2=default:RT_BVH_WIDTH=2,leaf3=default:RT_BVH_LEAF=3,leaf2=default:RT_BVH_LEAF=2,axes3=default:RT_BVH_AXES=3,bins32=default:RT_BVH_BINS=32,ax3b32=default:RT_BVH_AXES=3:RT_BVH_BINS=32,ax3l3=default:RT_BVH_AXES=3:RT_BVH_LEAF=3"
echo "== shadow"; timeout -k 10 250 python scripts/ab_variants.py --rounds 8 --variants "$V" > gpurun_out/abb_shadow.json 2> gpurun_out/abb_shadow.err; rc=$?; cat gpurun_out/abb_shadow.json; grep -c "identical=False" gpurun_out/abb_shadow.err; [ $rc -eq 0 ] || exit $rc
echo "== path"; timeout -k 10 250 python scripts/ab_variants.py --mode path --rounds 6 --variants "$V" > gpurun_out/abb_path.json 2> gpurun_out/abb_path.err; rc=$?; cat gpurun_out/abb_path.json; grep -c "identical=False" gpurun_out/abb_path.err; exit $rc
