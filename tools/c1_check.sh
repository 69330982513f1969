#!/bin/bash
# C1 (the device ctr triple): batch/parity tests, host time per section, the bench line at two step counts
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
if [ -z "$NOTEST" ]; then timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3; fi
timeout -k 10 200 python tools/host_prof.py 2>&1 | grep -v amdgpu
for s in 20 200; do
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline --steps $s 2>&1 | grep -v amdgpu | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, d['value'], d['ms_per_step'], json.dumps(d['host']))"
done
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline --no-profile 2>&1 | grep -v amdgpu | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('noprof', d['value'], d['ms_per_step'])"
