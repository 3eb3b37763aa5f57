# r04zg: the SAH build as one launch sequence -- its tests, the rebuild time, a bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zg
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_bvh_sah.py tests/test_gpu_bvh_build.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
grep -E "passed|failed|SAH build|tris," gpurun_out/${T}_pytest.log | tail -25
timeout -k 10 200 python3 bench.py --steps 200 --warmup 20 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json;j=json.load(open('gpurun_out/${T}_bench.json'));c=j['config'];print(j['value'],{k:c[k] for k in c if 'bvh' in k})"
