# r04j: path timeline (stamp image, local-sort node step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04j
echo "== path timeline"; timeout -k 10 150 python3 scripts/wave_timeline.py 1024 path > gpurun_out/${T}_path_timeline.json 2> gpurun_out/${T}_path_timeline.err; rc=$?; head -c 3000 gpurun_out/${T}_path_timeline.json; echo; [ $rc -eq 0 ] || exit $rc
echo "== path A/B adjacent pairs"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 8 --frames 10 --variants "x32=default,adj=adj" > gpurun_out/${T}_adj.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_adj.log; exit $rc
