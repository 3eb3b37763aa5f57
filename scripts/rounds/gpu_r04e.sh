# r04e: the setup sub-phases (split launches, kernel trace); A/B of the path
# tracer's quad lanes (16-pixel waves, 4 lanes per path) against the pairs
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04e
echo "== setup probe split"; RT_SETUP_SPLIT=1 RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_setup -o setup --output-format csv -- python3 scripts/setup_probe.py --moving 2 > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
echo "== ab path quad"; timeout -k 10 300 python scripts/ab_variants.py --mode path --rounds 8 --variants "default,quad=quad:RT_SPLIT_LOG=4,s16=default:RT_SPLIT_LOG=4" > gpurun_out/${T}_ab_quad.json 2> gpurun_out/${T}_ab_quad.err; rc=$?; cat gpurun_out/${T}_ab_quad.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_ab_quad.err; exit $rc; }
echo "== ab flat scalar"; timeout -k 10 250 python scripts/ab_variants.py --mode flat --size 256 --no-shadows --rounds 10 --variants "default,flatsc,flatsc128" > gpurun_out/${T}_ab_flat.json 2> gpurun_out/${T}_ab_flat.err; rc=$?; cat gpurun_out/${T}_ab_flat.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_ab_flat.err; exit $rc; }
