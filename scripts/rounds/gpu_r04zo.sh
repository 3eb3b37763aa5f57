# r04zo: SAH build tests, the 100k per-launch trace and the build probe (r04zo: per-wave BVH4 maxima; r04zq: workgroup-aggregated node ids for the small segments)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${T:-r04zo}
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bvh_sah.py tests/test_gpu_bvh_build.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }; tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 120 python3 scripts/sah_trace.py > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
grep -E "phase (1|6) |build_ms" gpurun_out/${T}_trace.log | tail -3
timeout -k 10 120 python3 scripts/sah_build_probe.py > gpurun_out/${T}_probe.json && cat gpurun_out/${T}_probe.json
