set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
tail -1 $O/tests.log
PSF_LIBRARY_VARIANT=tools/variants/trace/libpsf.so timeout -k 10 200 python tools/c1_trace.py > $O/trace.txt 2>&1
ROUNDS=4 CONFIGS="c1" EXTRA="--no-host-floor" timeout -k 10 900 bash tools/ab.sh r06x_c1 base head > $O/ab.log 2>&1
