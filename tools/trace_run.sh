#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for k in ${KINDS:-random codes}; do
  timeout -k 10 120 python tools/snappy_trace.py --run --name trace --kind $k --mib 128 2>&1 | grep -v amdgpu.ids || exit $?
done
