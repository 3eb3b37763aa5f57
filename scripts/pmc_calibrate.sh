# rocprofv3 FETCH_SIZE / WRITE_SIZE calibration on known-byte probes
# (skybox_rt_amd/lib/pmc_probe: 4-B/lane stores like the framebuffer store,
# 16-B/lane stores and loads, 64-B scalar-cache record loads), at the
# framebuffer's size (4 MiB) and past the L2 (64 MiB), one --pmc pass per
# counter; reduced by scripts/pmc_calibrate.py into $OUT (default
# profiles/pmc_calibration.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-cal}; mkdir -p gpurun_out/$TAG
for mib in 4 64; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c -d gpurun_out/$TAG/cal_${mib}_$c -o run --output-format csv -- \
      skybox_rt_amd/lib/pmc_probe $mib 6 > gpurun_out/$TAG/cal_${mib}_$c.log 2>&1 || { tail -5 gpurun_out/$TAG/cal_${mib}_$c.log; exit 1; }
  done
done
python3 scripts/pmc_calibrate.py gpurun_out/$TAG ${OUT:-profiles/pmc_calibration.json}
