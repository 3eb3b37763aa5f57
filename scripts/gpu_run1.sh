set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=skybox_rt_amd/lib
echo "== rtapp triangle" && timeout -k 10 120 $L/rtapp -t tests/golden/scenes/triangle.cgltrace -w 64 -h 64 -o gpurun_out/tri64.png -r tests/golden/draw3d/triangle_ref_64.png > gpurun_out/r1_rtapp_tri.log 2>&1; echo "rc=$?"; cat gpurun_out/r1_rtapp_tri.log | tail -5
echo "== rtapp tekkaman" && timeout -k 10 120 $L/rtapp -t tests/golden/scenes/tekkaman.cgltrace -w 1024 -h 1024 -S -n 20 -o gpurun_out/tk1024.png > gpurun_out/r1_rtapp_tk.log 2>&1; echo "rc=$?"; tail -5 gpurun_out/r1_rtapp_tk.log
