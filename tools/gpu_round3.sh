#!/bin/bash
# Round-3 GPU session: GPU tests, smoke, bench, host edge through the adapter,
# snappy throughput.  Each GPU step has its own time limit; a fault-like exit
# ends the script at once (tools/gpu_check.sh's step()).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_check.sh ${STEPS:-pytest smoke bench} || exit $?
if [ -n "$HOSTEDGE" ]; then
  timeout -k 10 600 python tools/host_edge_chain.py > gpurun_out/host_edge_chain.log 2>&1; rc=$?
  echo "host_edge rc=$rc"; tail -8 gpurun_out/host_edge_chain.log
  [ $rc -ge 124 ] && exit $rc
fi
if [ -n "$SNAPPY" ]; then
  timeout -k 10 300 python tools/bench_snappy.py --mib 128 --no-cpu > gpurun_out/bench_snappy.log 2>&1; rc=$?
  echo "bench_snappy rc=$rc"; tail -8 gpurun_out/bench_snappy.log
fi
exit 0
