# focused check of the fused FIXING_FLOAT-in-uncompress path: its tests, then
# kernel-trace stats of C5 + COMPRESSING
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-fused}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_snappy.py tests/test_gpu_batch.py tests/test_gpu_spill.py tests/test_gpu_adapter.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/prof_c5z.sh ${1:-fused}/prof
