set -o pipefail
# r05ah: run with profiles/r05/ab/r05ah_inkernel_signal.patch applied (VX_HIP_TAIL=2 =
# in-kernel completion); the patch was not kept, so at HEAD "sig" equals "done".
mkdir -p gpurun_out/r05ah
V="done=default:VX_HIP_TAIL=1,sig=default:VX_HIP_TAIL=2,ev=default:VX_HIP_TAIL=0"
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 8 --variants $V > gpurun_out/r05ah/shadow.json 2> gpurun_out/r05ah/shadow.err &&
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 8 --mode path --variants $V > gpurun_out/r05ah/path.json 2> gpurun_out/r05ah/path.err &&
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 8 --mode flat --no-shadows --variants $V > gpurun_out/r05ah/flat.json 2> gpurun_out/r05ah/flat.err &&
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 8 --bvh-walk --no-shadows --variants $V > gpurun_out/r05ah/bvh.json 2> gpurun_out/r05ah/bvh.err &&
cat gpurun_out/r05ah/*.json
