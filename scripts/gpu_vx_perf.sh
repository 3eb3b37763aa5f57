# vx_dump_perf classes from gfx950 counters (scripts/vx_perf.py) on the RT frame,
# the texture app and the raster pipeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/vx_perf; export TMPDIR=/tmp
for c in 1 2 3; do
  echo "== rt class $c"; timeout -k 10 400 python3 scripts/vx_perf.py --class $c --out gpurun_out/vx_perf/rt -- python3 scripts/prof_rt.py --frames 5 > gpurun_out/vx_perf/rt_class$c.txt 2>&1 || { cat gpurun_out/vx_perf/rt_class$c.txt; exit 1; }
  cat gpurun_out/vx_perf/rt_class$c.txt
done
echo "== tex class 3"; timeout -k 10 400 python3 scripts/vx_perf.py --class 3 --out gpurun_out/vx_perf/tex -- python3 scripts/prof_tex.py --case bilinear --frames 5 > gpurun_out/vx_perf/tex_class3.txt 2>&1 || exit 1
cat gpurun_out/vx_perf/tex_class3.txt
echo "== tex class 5"; timeout -k 10 400 python3 scripts/vx_perf.py --class 5 --out gpurun_out/vx_perf/tex -- python3 scripts/prof_tex.py --case point --frames 5 > gpurun_out/vx_perf/tex_class5.txt 2>&1 || exit 1
cat gpurun_out/vx_perf/tex_class5.txt
