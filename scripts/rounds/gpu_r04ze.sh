# r04ze: path A/B -- the quad code compiled in (no quad waves) vs the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04ze
echo "== path A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 10 --frames 10 --variants "base=default,quad1=quad1,q16=quad1:RT_QUAD_TILES=16" > gpurun_out/${T}_path.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_path.log; exit $rc
