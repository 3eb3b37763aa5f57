# r04zh: SAH build time against the launch grid (blocks of 256 threads per CU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=r04zh
: > gpurun_out/${T}.jsonl
for b in default 1 2 4 8; do
  if [ $b = default ]; then
    timeout -k 10 120 python3 scripts/sah_build_probe.py >> gpurun_out/${T}.jsonl || exit 1
  else
    VX_HIP_BLOCKS_PER_CU=$b timeout -k 10 120 python3 scripts/sah_build_probe.py >> gpurun_out/${T}.jsonl || exit 1
  fi
done
cat gpurun_out/${T}.jsonl
