# r03q: packed 16-bit Lerp8888 (RT_PK_LERP) -- parity of the shading paths,
# A/B on configs 3 and 4 against the 32-bit form
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03q FILES="tests/test_gpu_rt.py tests/test_gpu_pt.py tests/test_gpu_raster.py tests/test_gpu_tex.py" \
  AB_SHADOW="pk=default,nolerp=nolerp" AB_PATH="pk=default,nolerp=nolerp" \
  bash scripts/gpu_ab.sh
