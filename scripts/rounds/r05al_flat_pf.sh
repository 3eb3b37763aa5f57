set -o pipefail
# r05al: the flat block test's first rectangle round issued before the chunk
# map, each next round before the current round's candidates (RT_FLAT_BLK_PF)
mkdir -p gpurun_out/r05al
timeout -k 10 240 python3 -u scripts/ab_variants.py --rounds 16 --size 256 --mode flat --no-shadows --variants pf0,pf1=default > gpurun_out/r05al/flat.json 2> gpurun_out/r05al/flat.err &&
cat gpurun_out/r05al/flat.json
