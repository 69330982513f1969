#!/bin/bash
# snappy-focused GPU check: the COMPRESSING tests, then the codec throughput
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_bounded.py tests/test_gpu_fused.py tests/test_gpu_batch.py tests/test_gpu_spill.py tests/test_gpu_adapter.py tests/test_gpu_chain_adapter.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_snappy.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_snappy.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_snappy.py --mib 128 --no-cpu > gpurun_out/bench_snappy.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/bench_snappy.log; exit $rc
