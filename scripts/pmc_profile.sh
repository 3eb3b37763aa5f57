# rocprofv3 PMC record of one bench workload's kernel image: HBM traffic
# (FETCH_SIZE and WRITE_SIZE, separate passes) and the SQ / TCP / TCC counters
# that name the binding resource, one --pmc pass per counter group within the
# per-block limits (8 SQ, 4 TCC, 4 TCP, 2 GRBM), each over
# scripts/prof_rt.py (the product configuration: counters off), reduced by
# scripts/pmc_profile.py into gpurun_out/$TAG/pmc_<mode>.json over the timed
# image's own entry (vx_main_<image>).
# MODE = shadow (config 3, default), path (config 4), flat (config 2) or bvh
# (config 3 by BVH traversal only, image rt_bvh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-pmc}; mkdir -p gpurun_out/$TAG
MODE=${MODE:-shadow}
case $MODE in
  shadow) CO=rt_kernel.co; SZ=1024 ;;
  path)   CO=pt_kernel.co; SZ=1024 ;;  # RT_PT_QUEUE=1: CO=pt_primary.co,pt_queue.co
  flat)   CO=rt_flat.co;   SZ=256 ;;
  bvh)    CO=rt_bvh.co;    SZ=1024 ;;  # config 3 by BVH traversal (bench series "bvh_walk")
  shadow4096) CO=rt_kernel.co; SZ=4096 ;;  # config 5's frame on one GPU (bench series "strong_4096")
  *) echo "bad MODE $MODE"; exit 2 ;;
esac
# the record's mode / file: pmc_shadow_4096.json for the 4096^2 frame
PMODE=$MODE; RMODE=$MODE
[ $MODE = shadow4096 ] && { PMODE=shadow; RMODE=shadow_4096; }
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/$TAG/${MODE}_$name -o run --output-format csv -- python3 scripts/prof_rt.py --mode $PMODE --size $SZ --frames 10 > gpurun_out/$TAG/${MODE}_$name.log 2>&1
  local rc=$?
  echo "pmc $MODE $name rc=$rc"
  return $rc
}
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit $?
pass sq2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR || exit $?
pass sq3 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT || exit $?
pass mem TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit $?
python3 scripts/pmc_profile.py gpurun_out/$TAG $MODE $SZ $(echo $CO | sed 's#\([^,]*\)#skybox_rt_amd/lib/\1#g') gpurun_out/$TAG/pmc_$RMODE.json
