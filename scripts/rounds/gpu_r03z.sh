# r03z: shadow-list resolution on the nearest-first bounded lists (env
# RT_SLIST_N, no rebuild), configs 3 and 4
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03z AB_SHADOW="n256=default,n128=default:RT_SLIST_N=128,n512=default:RT_SLIST_N=512" \
  AB_PATH="n256=default,n512=default:RT_SLIST_N=512,n1024=default:RT_SLIST_N=1024" ROUNDS=10 \
  bash scripts/gpu_ab.sh
