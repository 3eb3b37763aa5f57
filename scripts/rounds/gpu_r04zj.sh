# r04zj: config 3 A/B -- empty blocks skip the list load (default now) vs not; + the layer record prefetched at wave start
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zj
timeout -k 10 300 python3 scripts/ab_variants.py --mode shadow --size 1024 --rounds 20 --frames 20 --variants "skip0=default,skip0off=skip0off,pflayer=pflayer" > gpurun_out/${T}_shadow.log 2>&1 || { tail -30 gpurun_out/${T}_shadow.log; exit 1; }
tail -1 gpurun_out/${T}_shadow.log
timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 8 --frames 8 --variants "skip0=default,skip0off=skip0off" > gpurun_out/${T}_path.log 2>&1 || { tail -30 gpurun_out/${T}_path.log; exit 1; }
tail -1 gpurun_out/${T}_path.log
