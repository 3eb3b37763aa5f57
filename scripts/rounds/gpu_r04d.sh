# r04d: per-sub-phase device times of the setup (RT_SETUP_SPLIT=1: every
# sub-phase its own launch) under a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04d
echo "== setup probe split"; RT_SETUP_SPLIT=1 RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_setup -o setup --output-format csv -- python3 scripts/setup_probe.py --moving 2 > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
