# HBM traffic of a bench workload: two separate rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE) over scripts/prof_rt.py, reduced by
# scripts/pmc_traffic.py into gpurun_out/$TAG/pmc_traffic[_<mode>].json.
# MODE = shadow (config 3, default), path (config 4) or flat (config 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-traffic}; mkdir -p gpurun_out/$TAG
MODE=${MODE:-shadow}
case $MODE in
  shadow) CO=rt_kernel.co; SZ=1024; SH=1; OUT=pmc_traffic.json ;;
  path)   CO=pt_kernel.co; SZ=1024; SH=1; OUT=pmc_traffic_path.json ;;
  flat)   CO=rt_flat.co;   SZ=256;  SH=0; OUT=pmc_traffic_flat.json ;;
  *) echo "bad MODE $MODE"; exit 2 ;;
esac
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/$TAG/fetch_$MODE -o run --output-format csv -- python3 scripts/prof_rt.py --mode $MODE --frames 10 > gpurun_out/$TAG/fetch_$MODE.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/$TAG/write_$MODE -o run --output-format csv -- python3 scripts/prof_rt.py --mode $MODE --frames 10 > gpurun_out/$TAG/write_$MODE.log 2>&1 || exit $?
python3 scripts/pmc_traffic.py gpurun_out/$TAG/fetch_$MODE gpurun_out/$TAG/write_$MODE gpurun_out/$TAG/$OUT $SZ $SZ $SH skybox_rt_amd/lib/$CO $MODE
