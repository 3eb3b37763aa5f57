set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03f FILES="tests/test_gpu_pt.py tests/test_gpu_blists.py tests/test_gpu_config5.py" \
  AB_PATH="bvh=default:RT_SHADOW_LISTS=0,lists=default,nosplit=default:RT_SPLIT_TILES=0,n128=default:RT_SLIST_N=128,n512=default:RT_SLIST_N=512" \
  bash scripts/gpu_ab.sh || exit $?
NS=2 STEPS=20 bash scripts/gpu_rehearsal.sh || exit $?
LIMS="1 16 256" bash scripts/lone_probe.sh || exit $?
timeout -k 10 200 python scripts/wave_timeline.py 1024 path > gpurun_out/lone/timeline_path.json 2> gpurun_out/lone/timeline_path.err
