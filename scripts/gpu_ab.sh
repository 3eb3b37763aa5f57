# Correctness of the default images on the named test files, then interleaved
# A/B timing of kernel variants: AB_SHADOW / AB_PATH variant lists
# (scripts/ab_variants.py).  TAG names the outputs under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-ab}
if [ -n "$FILES" ]; then
timeout -k 10 400 python -u -m pytest $FILES -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest.log | head; exit $rc; }
fi
if [ -n "$AB_SHADOW" ]; then timeout -k 10 300 python scripts/ab_variants.py --rounds ${ROUNDS:-8} --variants "$AB_SHADOW" > gpurun_out/${T}_shadow.json 2> gpurun_out/${T}_shadow.err || { tail -5 gpurun_out/${T}_shadow.err; exit 1; }; cat gpurun_out/${T}_shadow.json; fi
if [ -n "$AB_PATH" ]; then timeout -k 10 300 python scripts/ab_variants.py --mode path --rounds ${ROUNDS:-8} --variants "$AB_PATH" > gpurun_out/${T}_path.json 2> gpurun_out/${T}_path.err || { tail -5 gpurun_out/${T}_path.err; exit 1; }; cat gpurun_out/${T}_path.json; fi
if [ -n "$AB_FLAT" ]; then timeout -k 10 300 python scripts/ab_variants.py --mode flat --size 256 --no-shadows --rounds ${ROUNDS:-8} --variants "$AB_FLAT" > gpurun_out/${T}_flat.json 2> gpurun_out/${T}_flat.err || { tail -5 gpurun_out/${T}_flat.err; exit 1; }; cat gpurun_out/${T}_flat.json; fi
if [ -n "$AB_BVH" ]; then timeout -k 10 300 python scripts/ab_variants.py --bvh-walk --rounds ${ROUNDS:-8} --variants "$AB_BVH" > gpurun_out/${T}_bvh.json 2> gpurun_out/${T}_bvh.err || { tail -5 gpurun_out/${T}_bvh.err; exit 1; }; cat gpurun_out/${T}_bvh.json; fi
