# r03h: path tracer in two kernels (pt_primary + pt_queue) -- parity tests,
# then A/B: paths per pt_queue wave, the one-kernel form, list resolution;
# config 3: list resolution, scalar work-order load
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03h FILES="tests/test_gpu_pt.py tests/test_gpu_blists.py tests/test_gpu_rt.py tests/test_gpu_bvh_sah.py" \
  AB_PATH="q64=default,q32=default:RT_PQ_LANES=32,q16=default:RT_PQ_LANES=16,one=default:RT_PT_QUEUE=0,q64n512=default:RT_SLIST_N=512" \
  AB_SHADOW="base=default,n256=default:RT_SLIST_N=256,osl" \
  bash scripts/gpu_ab.sh
