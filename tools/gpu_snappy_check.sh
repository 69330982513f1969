#!/bin/bash
# The snappy GPU tests (compress, uncompress, fused decode, bounded waits) and
# tools/bench_snappy.py on every payload (compress + uncompress), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/snappy_check; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_bounded.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > gpurun_out/snappy_check/tests.log 2>&1 || { tail -30 gpurun_out/snappy_check/tests.log; exit 1; }
tail -1 gpurun_out/snappy_check/tests.log
timeout -k 10 300 python3 tools/bench_snappy.py --mib 128 --no-cpu --reps 3 > gpurun_out/snappy_check/bench.log 2>&1 || { tail -5 gpurun_out/snappy_check/bench.log; exit 1; }
grep payload gpurun_out/snappy_check/bench.log
