# r04y: path A/B -- branch-free leaf tests in the pair walk
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04y
echo "== path A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 10 --frames 10 --variants "base=default,leafbf=leafbf,listbf=listbf" > gpurun_out/${T}_path.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_path.log; exit $rc
