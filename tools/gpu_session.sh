set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06d2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_fused.py tests/test_gpu_c4_batch.py tests/test_gpu_timed_sizes.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
ROUNDS=3 CONFIGS="c3 c4 c5 c1 c2" EXTRA="--no-host-floor" timeout -k 10 1000 bash tools/ab.sh r06d2_dec base head > $O/ab.log 2>&1
