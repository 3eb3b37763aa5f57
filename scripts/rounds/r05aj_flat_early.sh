set -o pipefail
# r05aj: the flat image without the second barrier when no shadow rays
# (RT_FLAT_EARLY_OUT), alone and with two block-test rounds in flight
mkdir -p gpurun_out/r05aj
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 12 --size 256 --mode flat --no-shadows --variants eo0,eo1=default,fu2,eo_u2 > gpurun_out/r05aj/flat.json 2> gpurun_out/r05aj/flat.err &&
cat gpurun_out/r05aj/flat.json
