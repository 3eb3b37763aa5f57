# Run the given GPU test files (FILES="tests/a.py tests/b.py") with output to
# gpurun_out/${TAG}.log.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-files}
timeout -k 10 ${LIMIT:-500} python -u -m pytest $FILES -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${T}.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert|launches" gpurun_out/${T}.log | tail -40; exit $rc
