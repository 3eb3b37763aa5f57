# r03l: config-4 isolation probes on the cooperative image -- the first n
# tiles of the work order alone (RT_TILE_LIMIT), 16 pixels per split wave,
# no split tiles
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r03l \
  AB_PATH="coop=default,lim1=default:RT_TILE_LIMIT=1,lim16=default:RT_TILE_LIMIT=16,lim64=default:RT_TILE_LIMIT=64,lim200=default:RT_TILE_LIMIT=200,lim400=default:RT_TILE_LIMIT=400,s4=default:RT_SPLIT_LOG=4,nosplit=default:RT_SPLIT_TILES=0,nc1=nocoop:RT_TILE_LIMIT=1" \
  bash scripts/gpu_ab.sh
