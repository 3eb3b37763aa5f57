# r04x: config-3 A/B -- the first layer record prefetched at wave start
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04x
echo "== shadow A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --size 1024 --rounds 10 --frames 20 --variants "base=default,lpre=lpre" > gpurun_out/${T}_shadow.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_shadow.log; exit $rc
