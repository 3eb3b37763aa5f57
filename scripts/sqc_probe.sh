set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/sqc
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/sqc/avail.txt 2>&1; echo list rc=$?
grep -o 'SQC_[A-Z_0-9]*' gpurun_out/sqc/avail.txt | sort -u > gpurun_out/sqc/sqc_names.txt; cat gpurun_out/sqc/sqc_names.txt | tr '\n' ' '
timeout -s KILL 90 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES_DUPLICATE -d gpurun_out/sqc/shadow -o run --output-format csv -- python3 scripts/prof_rt.py --mode shadow --frames 10 > gpurun_out/sqc/shadow.log 2>&1; echo pass rc=$?
