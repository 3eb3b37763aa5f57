# Round 5 GPU calls.  STEPS = space-separated list, run in order, the first
# failure ends the call; TAG names the outputs under gpurun_out/.
#   tests   pytest -m gpu (FILES= to restrict to some test files)
#   bench   python bench.py --workload W $BENCH_ARGS for W in WORKLOADS (-> ${TAG}_bench_W.json)
#   smoke   __graft_entry__.smoke()
#   host    scripts/host_overhead.py (start / wait / kernel split of a synchronous frame)
#   ab      scripts/gpu_ab.sh with AB_SHADOW / AB_PATH / AB_FLAT variant lists
#   prof    rocprofv3 --kernel-trace --stats of bench.py --workload W --no-cpu-baseline $BENCH_ARGS
#   pmc     scripts/pmc_profile.sh for MODES (default: shadow)
#   timeline scripts/wave_timeline.py 1024 <mode> for TL_MODES (shadow, bvh, path; make diag)
#   abtree  bench.py here against abtree/bench.py (another build), alternated ABTREE_ROUNDS times
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r05}
for s in ${STEPS:-tests bench}; do
  echo "== $s"
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
        > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log
      [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_gpu.log | head -20; exit $rc; } ;;
    bench)
      for w in ${WORKLOADS:-shadow}; do
        timeout -k 10 400 python bench.py --workload $w $BENCH_ARGS > gpurun_out/${T}_bench_$w.json \
          2> gpurun_out/${T}_bench_$w.err || { tail -5 gpurun_out/${T}_bench_$w.err; exit 1; }
        python3 -c "import json;j=json.load(open('gpurun_out/${T}_bench_$w.json'));c=j['config'];print('$w',j['value'],j['ms_per_step'],c['kernel_ms'],c.get('sync_ms_per_step'),j['roofline']['frac'])"
      done ;;
    smoke)
      timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/${T}_smoke.log 2>&1 \
        || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }; tail -1 gpurun_out/${T}_smoke.log ;;
    host)
      timeout -k 10 120 python scripts/host_overhead.py > gpurun_out/${T}_host.json 2> gpurun_out/${T}_host.err \
        || { tail -5 gpurun_out/${T}_host.err; exit 1; }; cat gpurun_out/${T}_host.json ;;
    ab)
      TAG=${T}_ab FILES= bash scripts/gpu_ab.sh || exit 1 ;;
    prof)
      for w in ${WORKLOADS:-shadow}; do
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$w -o ${T}_$w --output-format csv \
          -- python3 bench.py --workload $w --no-cpu-baseline $BENCH_ARGS > gpurun_out/${T}_prof_$w.log 2>&1 \
          || { tail -5 gpurun_out/${T}_prof_$w.log; exit 1; }
      done ;;
    pmc)
      for m in ${MODES:-shadow}; do
        MODE=$m TAG=${T}_pmc bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc_$m.log 2>&1 \
          || { tail -5 gpurun_out/${T}_pmc_$m.log; exit 1; }
      done ;;
    timeline)
      for m in ${TL_MODES:-shadow}; do
        if [ $m = flat ]; then tl="scripts/flat_timeline.py 256"; else tl="scripts/wave_timeline.py 1024 $m"; fi
        timeout -k 10 180 python $tl > gpurun_out/${T}_timeline_$m.json \
          2> gpurun_out/${T}_timeline_$m.err || { tail -5 gpurun_out/${T}_timeline_$m.err; exit 1; }
        head -c 1500 gpurun_out/${T}_timeline_$m.json; echo
      done ;;
    abtree)
      # whole-bench A/B against another build staged in abtree/ (the
      # previous commit's tree: a driver ABI change cannot be A/B'd as
      # kernel-image variants), alternated ABTREE_ROUNDS times on this box
      for i in $(seq ${ABTREE_ROUNDS:-2}); do
        for side in new old; do
          b=bench.py; [ $side = old ] && b=abtree/bench.py
          timeout -k 10 300 python $b --no-cpu-baseline $BENCH_ARGS > gpurun_out/${T}_abtree_${side}_$i.json \
            2> gpurun_out/${T}_abtree_${side}_$i.err || { tail -5 gpurun_out/${T}_abtree_${side}_$i.err; exit 1; }
          python3 -c "import json;j=json.load(open('gpurun_out/${T}_abtree_${side}_$i.json'));c=j['config'];s=j.get('series',{});print('$side',$i,c['kernel_ms'],*[(k,v.get('kernel_ms'),v.get('ms_per_step')) for k,v in s.items()])"
        done
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
