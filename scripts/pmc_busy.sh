# Busy counters of the memory / scalar pipelines for one workload's kernel
# image (which shared pipeline the resident waves queue
# on): TA / TD busy cycles, the scalar data cache, the instruction cache,
# vector-memory and scalar instruction activity -- each pass a few counters
# of one block (within the per-block limits), only names this rocprofv3
# lists, each under its own kill timeout; reduced by scripts/pmc_busy.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-busy}; MODE=${MODE:-shadow}; mkdir -p gpurun_out/$TAG
timeout -s KILL 60 rocprofv3 -L > gpurun_out/$TAG/counters.txt 2>&1 || true
has() { grep -qw "$1" gpurun_out/$TAG/counters.txt; }
pass() {  # name, counters... (the ones listed)
  local name=$1; shift; local cs=()
  for c in "$@"; do has "$c" && cs+=("$c"); done
  [ ${#cs[@]} -eq 0 ] && { echo "pass $name: none listed"; return 0; }
  echo "pass $name: ${cs[*]}"
  timeout -s KILL 60 rocprofv3 --pmc "${cs[@]}" -d gpurun_out/$TAG/${MODE}_$name -o run --output-format csv \
    -- python3 scripts/prof_rt.py --mode $MODE --frames 10 > gpurun_out/$TAG/${MODE}_$name.log 2>&1
}
pass ta GRBM_GUI_ACTIVE TA_TA_BUSY_sum TD_TD_BUSY_sum || exit $?
pass tastall TA_BUFFER_WAVEFRONTS_sum TA_FLAT_WAVEFRONTS_sum || exit $?
pass tcp TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum || exit $?
pass sqc SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_ICACHE_MISSES || exit $?
pass sqi SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit $?
python3 scripts/pmc_busy.py gpurun_out/$TAG $MODE > gpurun_out/$TAG/busy_$MODE.json
