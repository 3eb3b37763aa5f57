# PMC passes over one tex case (scripts/prof_tex.py); CASE=point|bilinear|trilinear
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-pmctex}; CASE=${CASE:-bilinear}; mkdir -p gpurun_out/$TAG
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" -d gpurun_out/$TAG/$name -o run --output-format csv -- python3 scripts/prof_tex.py --case $CASE --frames 10 > gpurun_out/$TAG/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  return 0
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR
run p4 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
run p5 FETCH_SIZE
run p6 WRITE_SIZE
run p7 TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum SQ_INSTS_FLAT
run p8 TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
python3 scripts/pmc_summary.py gpurun_out/$TAG > gpurun_out/$TAG/summary.txt; cat gpurun_out/$TAG/summary.txt
