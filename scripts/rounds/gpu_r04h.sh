# r04h: full GPU suite with shadow lists at N = 128 and the interleaved,
# paired two-level flat scan; flat A/B; setup launch trace (non-split)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04h
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
echo "== flat A/B"; timeout -k 10 200 python3 scripts/ab_variants.py --mode flat --no-shadows --size 256 --rounds 10 --frames 20 --variants "t256=default,onelevel=flat1,t512=flat_t512,t1024=flat_t1024" > gpurun_out/${T}_flat.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_flat.log; [ $rc -eq 0 ] || exit $rc
echo "== flat timeline"; timeout -k 10 120 python3 scripts/flat_timeline.py 256 > gpurun_out/${T}_flat_timeline.json 2> gpurun_out/${T}_flat_timeline.err; rc=$?; cat gpurun_out/${T}_flat_timeline.json; echo; [ $rc -eq 0 ] || exit $rc
echo "== setup trace"; RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_strace -o setup --output-format csv -- python3 scripts/setup_probe.py --moving 3 > gpurun_out/${T}_strace.json 2> gpurun_out/${T}_strace.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_strace.err; exit $rc; }
python3 -c "
import json;d=json.load(open('gpurun_out/${T}_strace.json'))
print(' '.join('%s=%s'%(x['tag'],x.get('configure_ms',x.get('set_light_wait_ms'))) for x in d))"
