# r04zk: per-launch times of the SAH build sequence (RT_SAH_TRACE: each launch its own timed run), 100k triangles
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zk
timeout -k 10 120 python3 scripts/sah_trace.py > gpurun_out/${T}.log 2>&1 || { tail -20 gpurun_out/${T}.log; exit 1; }
sed -n '/second build/,$p' gpurun_out/${T}.log
