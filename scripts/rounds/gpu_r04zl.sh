# r04zl: SAH build (4 triangles per thread in the workgroup loops, bit-path BVH4 membership, merged emit atomics, unrolled scan): tests, trace, probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zl
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_bvh_sah.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
grep -E "passed|failed|SAH build|tris," gpurun_out/${T}_pytest.log | tail -20
timeout -k 10 120 python3 scripts/sah_trace.py > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
sed -n '/second build/,$p' gpurun_out/${T}_trace.log | tr '\n' ' '; echo
timeout -k 10 120 python3 scripts/sah_build_probe.py > gpurun_out/${T}_probe.json && cat gpurun_out/${T}_probe.json
