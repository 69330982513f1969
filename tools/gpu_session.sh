set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06p2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_stored.py tests/test_gpu_batch.py tests/test_gpu_timed_sizes.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
ROUNDS=4 CONFIGS="c5z c5zm" EXTRA="--no-host-floor" timeout -k 10 900 bash tools/ab.sh r06p2_c5z base head > $O/ab.log 2>&1
