# r04f: setup after the LINK-side leaf covers and the 1024-workgroup grid:
# the setup / light / list tests, then per-sub-phase times (split launches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04f
echo "== pytest setup"; timeout -k 10 300 python -u -m pytest tests/test_gpu_light.py tests/test_gpu_setup.py tests/test_gpu_blists.py tests/test_gpu_bvh_walk.py tests/test_gpu_edge_kat.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest_setup.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_pytest_setup.log; grep "cold configure" gpurun_out/${T}_pytest_setup.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${T}_pytest_setup.log | head -20; exit $rc; }
echo "== setup probe"; timeout -k 10 200 python3 scripts/setup_probe.py > gpurun_out/${T}_setup.json 2> gpurun_out/${T}_setup.err; rc=$?; python3 -c "
import json;d=json.load(open('gpurun_out/${T}_setup.json'))
for x in d: print(x['tag'], x.get('configure_ms'), x.get('set_light_wait_ms'), x.get('launches'))"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_setup.err; exit $rc; }
echo "== setup probe split"; RT_SETUP_SPLIT=1 RT_SETUP_TRACE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${T}_split -o setup --output-format csv -- python3 scripts/setup_probe.py --moving 2 > gpurun_out/${T}_split.json 2> gpurun_out/${T}_split.err; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_split.err; exit $rc; }
echo "== quad tiers (path, config 4)"; timeout -k 10 300 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 6 --frames 10 --variants "base=default,q0=quad,q8=quad:RT_QUAD_TILES=8,q16=quad:RT_QUAD_TILES=16,q32=quad:RT_QUAD_TILES=32,q64=quad:RT_QUAD_TILES=64" > gpurun_out/${T}_quad.log 2>&1; rc=$?; tail -12 gpurun_out/${T}_quad.log; [ $rc -eq 0 ] || exit $rc
echo "== flat grid (config 2)"; timeout -k 10 200 python3 scripts/ab_variants.py --mode flat --no-shadows --size 256 --rounds 8 --frames 20 --variants "base=default,g4=default:VX_HIP_BLOCKS_PER_CU=4,g6=default:VX_HIP_BLOCKS_PER_CU=6,g8=default:VX_HIP_BLOCKS_PER_CU=8" > gpurun_out/${T}_flatgrid.log 2>&1; rc=$?; tail -6 gpurun_out/${T}_flatgrid.log; [ $rc -eq 0 ] || exit $rc
echo "== flat timeline"; timeout -k 10 120 python3 scripts/flat_timeline.py 256 > gpurun_out/${T}_flat_timeline.json 2> gpurun_out/${T}_flat_timeline.err; rc=$?; cat gpurun_out/${T}_flat_timeline.json; [ $rc -eq 0 ] || exit $rc
echo "== bvh occupancy (config 3 BVH form)"; timeout -k 10 200 python3 scripts/ab_variants.py --bvh-walk --size 1024 --rounds 8 --frames 20 --variants "base=default,w5=bvh_w5,w6=bvh_w6,w8=bvh_w8" > gpurun_out/${T}_bvh_occ.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_bvh_occ.log; [ $rc -eq 0 ] || exit $rc
echo "== bvh timeline"; timeout -k 10 120 python3 scripts/wave_timeline.py 1024 bvh > gpurun_out/${T}_bvh_timeline.json 2> gpurun_out/${T}_bvh_timeline.err; rc=$?; head -c 3000 gpurun_out/${T}_bvh_timeline.json; echo; [ $rc -eq 0 ] || exit $rc
echo "== path timeline (ptstamp)"; timeout -k 10 150 python3 scripts/wave_timeline.py 1024 path > gpurun_out/${T}_path_timeline.json 2> gpurun_out/${T}_path_timeline.err; rc=$?; head -c 3000 gpurun_out/${T}_path_timeline.json; echo; [ $rc -eq 0 ] || exit $rc
for v in default xcd; do
  kd=skybox_rt_amd/lib; [ $v = default ] || kd=skybox_rt_amd/lib/variants/$v
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${T}_xcd_$v/fetch -o run --output-format csv -- python3 scripts/prof_rt.py --mode shadow --frames 10 --kernel-dir $kd > gpurun_out/${T}_xcd_${v}_fetch.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum -d gpurun_out/${T}_xcd_$v/mem -o run --output-format csv -- python3 scripts/prof_rt.py --mode shadow --frames 10 --kernel-dir $kd > gpurun_out/${T}_xcd_${v}_mem.log 2>&1 || exit $?
  echo "xcd pmc $v ok"
done
