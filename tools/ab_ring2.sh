# K4 occupancy A/B: tools/variants/{cur,lb8,old}, sorted keys + zeros + stored payloads, twice
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ring2}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_fused.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in cur lb8 old; do
  echo "== $v"
  PSF_LIBRARY_VARIANT=$PWD/tools/variants/$v/libpsf.so timeout -k 10 200 python -u tools/bench_snappy.py --mib 128 --no-cpu 2>&1 | grep payload | cut -c1-200 || exit 1
done
done
