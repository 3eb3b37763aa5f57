# HBM traffic of the bench workload: two separate rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE) over scripts/prof_rt.py, reduced by
# scripts/pmc_traffic.py into gpurun_out/$TAG/pmc_traffic.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-traffic}; mkdir -p gpurun_out/$TAG
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$TAG/fetch -o run --output-format csv -- python3 scripts/prof_rt.py --frames 10 > gpurun_out/$TAG/fetch.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$TAG/write -o run --output-format csv -- python3 scripts/prof_rt.py --frames 10 > gpurun_out/$TAG/write.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/$TAG/fetch gpurun_out/$TAG/write gpurun_out/$TAG/pmc_traffic.json 1024 1024 1 skybox_rt_amd/lib/rt_kernel.co
