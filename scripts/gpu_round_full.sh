set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-full} bash scripts/gpu_round.sh || exit $?
echo "== timeline shadow"; timeout -k 10 200 python scripts/wave_timeline.py 1024 > gpurun_out/${TAG:-full}_timeline_shadow.json 2> gpurun_out/${TAG:-full}_timeline_shadow.err || exit 1
echo "== timeline path"; timeout -k 10 200 python scripts/wave_timeline.py 1024 path > gpurun_out/${TAG:-full}_timeline_path.json 2> gpurun_out/${TAG:-full}_timeline_path.err || exit 1
echo "== bvh build bench"; timeout -k 10 300 python scripts/bench_bvh_build.py > gpurun_out/${TAG:-full}_bvh_build_bench.jsonl 2> gpurun_out/${TAG:-full}_bvh_build_bench.err || exit 1
cat gpurun_out/${TAG:-full}_bvh_build_bench.jsonl
