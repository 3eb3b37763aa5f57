# r03x: shadow lists ordered nearest-to-the-light first with the scan bounded
# by the segment's length -- parity (lists, frames, counts), A/B vs the
# unbounded scan on configs 3 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03x FILES="tests/test_gpu_blists.py tests/test_gpu_rt.py tests/test_gpu_pt.py tests/test_gpu_setup.py" \
  AB_SHADOW="bound=default,nobound=nobound" AB_PATH="bound=default,nobound=nobound" ROUNDS=10 \
  bash scripts/gpu_ab.sh
