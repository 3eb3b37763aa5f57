# r03v: config 4 with / without the counter gate (VX_ROWS_GATE) and config 3
# with 128-thread workgroups, 16 interleaved rounds each
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03v AB_PATH="gate=default,nogate=ptnogate" AB_SHADOW="base=default,b128=b128" ROUNDS=16 \
  bash scripts/gpu_ab.sh
