# r03u: the r03t A/B (128-thread workgroups, layers first), then the full
# round on the shipped images (tests, smoke, PMC records, bench lines,
# rocprof summaries)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python scripts/ab_variants.py --rounds 12 --variants "base=default,b128=b128,lfirst=lfirst,b128lf=b128lf" > gpurun_out/r03u_ab_shadow.json 2> gpurun_out/r03u_ab_shadow.err || { tail -5 gpurun_out/r03u_ab_shadow.err; exit 1; }
cat gpurun_out/r03u_ab_shadow.json
TAG=r03u bash scripts/gpu_round.sh
