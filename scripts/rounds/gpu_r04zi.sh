# r04zi: config 3 wave timeline (stamp image): where a background wave's time goes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zi
timeout -k 10 120 python3 scripts/wave_timeline.py 1024 > gpurun_out/${T}_timeline.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 1; }
cat gpurun_out/${T}_timeline.json
