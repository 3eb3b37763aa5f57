# r04zf: path A/B -- every wave's paths on compacted lane pairs (PT_COOP_ALL, 4 waves per SIMD) vs the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zf
echo "== path A/B"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 10 --frames 10 --variants "base=default,coopall=coopall,coopall3=coopall3,coopall_ns=coopall:RT_SPLIT_TILES=0" > gpurun_out/${T}_path.log 2>&1 || { tail -30 gpurun_out/${T}_path.log; exit 1; }
tail -1 gpurun_out/${T}_path.log
echo "== path A/B, no shadow lists"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 6 --frames 6 --variants "base_nl=default:RT_SHADOW_LISTS=0,coopall_nl=coopall:RT_SHADOW_LISTS=0" > gpurun_out/${T}_nl.log 2>&1 || { tail -30 gpurun_out/${T}_nl.log; exit 1; }
tail -1 gpurun_out/${T}_nl.log
