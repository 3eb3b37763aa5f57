# r04l: path A/B -- leaf triangles interleaved over the pair, normal carried from the hit
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04l
echo "== path A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 8 --frames 10 --variants "base=default,il=il,nrm=nrm,ilnrm=ilnrm" > gpurun_out/${T}_path.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_path.log; exit $rc
