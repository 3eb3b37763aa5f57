# Isolation probes for config 3: per-wave phase stamps (RT_STAMPS image,
# incl. the packet walks' record-load wait cycles) for the full frame and with
# only the heaviest tile(s) rendered (RT_TILE_LIMIT).  gpurun_out/lone/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lone
timeout -k 10 200 python scripts/wave_timeline.py 1024 > gpurun_out/lone/timeline_full.json 2> gpurun_out/lone/timeline_full.err || exit 1
for n in ${LIMS:-1 16}; do
RT_TILE_LIMIT=$n timeout -k 10 200 python scripts/wave_timeline.py 1024 > gpurun_out/lone/timeline_lim$n.json 2> gpurun_out/lone/timeline_lim$n.err || exit 1
done
