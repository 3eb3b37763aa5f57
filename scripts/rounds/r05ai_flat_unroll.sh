set -o pipefail
# r05ai: the flat image's block test with 2 / 4 rounds of rectangle words in flight
mkdir -p gpurun_out/r05ai
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 12 --size 256 --mode flat --no-shadows --variants base=default,fu2,fu4 > gpurun_out/r05ai/flat.json 2> gpurun_out/r05ai/flat.err &&
cat gpurun_out/r05ai/flat.json
