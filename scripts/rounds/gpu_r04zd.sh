# r04zd: the driver's round-end entry points: smoke() on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04zd_smoke.log 2>&1; rc=$?; tail -5 gpurun_out/r04zd_smoke.log; exit $rc
