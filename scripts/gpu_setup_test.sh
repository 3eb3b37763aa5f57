set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_setup.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/setup1.log 2>&1; rc=$?; tail -25 gpurun_out/setup1.log; exit $rc
