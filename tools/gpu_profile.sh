#!/bin/bash
# Profiling session for profiles/: kernel-trace stats of the bench command and
# separate PMC passes (FETCH_SIZE, WRITE_SIZE) -- counters never combined with
# any tracing domain other than the kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof gpurun_out/pmc
TAG=${1:-r01}
ARGS=${BENCH_ARGS:---no-cpu-baseline --steps 20 --warmup 3}
set -o pipefail
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $TAG -- python3 bench.py $ARGS > gpurun_out/prof/$TAG.bench.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- python3 bench.py $ARGS --no-profile > gpurun_out/pmc/${TAG}_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- python3 bench.py $ARGS --no-profile > gpurun_out/pmc/${TAG}_write.log 2>&1 || exit $?
ls -la gpurun_out/prof gpurun_out/pmc
