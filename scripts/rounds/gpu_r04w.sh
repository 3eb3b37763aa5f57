# r04w: config-3 wave timeline (stamp image) on the current images
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04w
echo "== shadow timeline"; timeout -k 10 150 python3 scripts/wave_timeline.py 1024 > gpurun_out/${T}_shadow_timeline.json 2> gpurun_out/${T}_shadow_timeline.err; rc=$?; head -c 4000 gpurun_out/${T}_shadow_timeline.json; echo; exit $rc
