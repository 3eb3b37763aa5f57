# r03t: config 3 -- 128-thread workgroups and the screen layers resolved
# before the primary pass (RT_LAYERS_FIRST); parity of the RT images
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03t FILES="tests/test_gpu_rt.py tests/test_gpu_setup.py tests/test_gpu_blists.py" \
  AB_SHADOW="base=default,b128=b128,lfirst=lfirst,b128lf=b128lf" ROUNDS=12 \
  bash scripts/gpu_ab.sh
