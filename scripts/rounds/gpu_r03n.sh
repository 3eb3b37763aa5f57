# r03n: config-4 wave timeline of the lane-pair image (ptstamp variant):
# the full frame and the 16 heaviest tiles alone (RT_TILE_LIMIT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/r03n
timeout -k 10 200 python scripts/wave_timeline.py 1024 path > gpurun_out/r03n/timeline_path_full.json 2> gpurun_out/r03n/timeline_path_full.err || exit 1
RT_TILE_LIMIT=16 timeout -k 10 200 python scripts/wave_timeline.py 1024 path > gpurun_out/r03n/timeline_path_lim16.json 2> gpurun_out/r03n/timeline_path_lim16.err || exit 1
cat gpurun_out/r03n/timeline_path_lim16.json
