#!/bin/bash
# rocprofv3 kernel stats of the snappy codec on one payload (default: FIXING_FLOAT codes)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=${1:-ff_codes_nb1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_snappy_$P -o run -- python3 tools/bench_snappy.py --mib 128 --no-cpu --only $P > gpurun_out/prof_snappy_$P.log 2>&1 || exit $?
f=$(find gpurun_out/prof_snappy_$P -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -20
