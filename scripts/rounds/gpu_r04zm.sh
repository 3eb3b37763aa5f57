# r04zm: config 4 launch-shape sweep (env only): grid per CU, 16-pixel split waves; SAH build at 512 / 1024-thread workgroups
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zm
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bvh_sah.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }; tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 400 python3 scripts/ab_variants.py --mode path --size 1024 --rounds 10 --frames 10 --variants "base=default,g64=default:VX_HIP_BLOCKS_PER_CU=64,g96=default:VX_HIP_BLOCKS_PER_CU=96,g192=default:VX_HIP_BLOCKS_PER_CU=192,g256=default:VX_HIP_BLOCKS_PER_CU=256,sl4=default:RT_SPLIT_LOG=4" > gpurun_out/${T}_path.log 2>&1 || { tail -30 gpurun_out/${T}_path.log; exit 1; }
tail -1 gpurun_out/${T}_path.log
for k in sah512 sah1024; do
  timeout -k 10 120 python3 scripts/sah_build_probe.py --kdir skybox_rt_amd/lib/variants/$k > gpurun_out/${T}_$k.json || exit 1; cat gpurun_out/${T}_$k.json
done
timeout -k 10 120 python3 scripts/sah_build_probe.py > gpurun_out/${T}_sahbase.json && cat gpurun_out/${T}_sahbase.json
