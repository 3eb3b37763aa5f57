# r03r: shading uniform waves from scalar-loaded records (RT_SHADE_UNIFORM)
# and no counter sums / block barriers with counters off (VX_ROWS_ALWAYS=0)
# -- parity of the RT / PT / flat images and the counters, A/B on configs 3, 4, 2
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03r FILES="tests/test_gpu_rt.py tests/test_gpu_pt.py tests/test_gpu_flat.py tests/test_vx_perf.py" \
  AB_SHADOW="both=default,noshu=noshu,nogate=nogate,osl=osl" AB_PATH="both=default,noshu=noshu,nogate=nogate,osl=osl" \
  AB_FLAT="both=default,noshu=noshu,nogate=nogate" \
  bash scripts/gpu_ab.sh
