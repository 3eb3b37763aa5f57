# r03s: config 3 workgroup size and occupancy re-measured after the counter
# gate (finished waves retire on their own now)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03s AB_SHADOW="base=default,b64=b64,b128=b128,w8=w8,w6=w6" \
  AB_FLAT="base=default,b64=b64,b128=b128" \
  bash scripts/gpu_ab.sh
