# r04g: full GPU suite after the two-level flat scan, the partitioned setup
# launches and the edge KAT; setup probes (partition on/off, N=128 lists);
# A/Bs: flat scan / workgroup size, shadow-list resolution (config 3 and 4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04g
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
for v in "part:" "nopart:RT_SETUP_PART=0" "n128:RT_SLIST_N=128"; do
  n=${v%%:*}; e=${v#*:}
  echo "== setup probe $n"; env $e timeout -k 10 200 python3 scripts/setup_probe.py > gpurun_out/${T}_setup_$n.json 2> gpurun_out/${T}_setup_$n.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup_$n.err; exit $rc; }
  python3 -c "
import json;d=json.load(open('gpurun_out/${T}_setup_$n.json'))
print(' '.join('%s=%s'%(x['tag'],x.get('configure_ms',x.get('set_light_wait_ms'))) for x in d))"
done
echo "== flat A/B"; timeout -k 10 200 python3 scripts/ab_variants.py --mode flat --no-shadows --size 256 --rounds 8 --frames 20 --variants "block=default,onelevel=flat1,t64=flat_t64,t128=flat_t128,t512=flat_t512" > gpurun_out/${T}_flat.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_flat.log; [ $rc -eq 0 ] || exit $rc
echo "== flat timeline"; timeout -k 10 120 python3 scripts/flat_timeline.py 256 > gpurun_out/${T}_flat_timeline.json 2> gpurun_out/${T}_flat_timeline.err; rc=$?; cat gpurun_out/${T}_flat_timeline.json; echo; [ $rc -eq 0 ] || exit $rc
echo "== slist N A/B config 3"; timeout -k 10 200 python3 scripts/ab_variants.py --size 1024 --rounds 8 --frames 20 --variants "n256=default,n128=default:RT_SLIST_N=128,n64=default:RT_SLIST_N=64" > gpurun_out/${T}_sn3.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_sn3.log; [ $rc -eq 0 ] || exit $rc
echo "== slist N A/B config 4"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 6 --frames 10 --variants "n256=default,n128=default:RT_SLIST_N=128" > gpurun_out/${T}_sn4.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_sn4.log; exit $rc
