# A/B of the fragment decoder's 8 KiB LDS output ring (K4): the snappy / fused /
# bounded tests, then tools/bench_snappy.py on every payload with the current
# build and with tools/variants/old (the 64 KiB LDS fragment), twice each,
# and a kernel trace of sorted keys.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ring}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_fused.py tests/test_gpu_bounded.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in new old new old; do
  echo "== $v"
  if [ $v = old ]; then export PSF_LIBRARY_VARIANT=$PWD/tools/variants/old/libpsf.so; else unset PSF_LIBRARY_VARIANT; fi
  timeout -k 10 200 python -u tools/bench_snappy.py --mib 128 --no-cpu 2>&1 | grep payload || exit 1
done
unset PSF_LIBRARY_VARIANT
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/tools/bench_snappy.py --mib 128 --no-cpu --only sorted_keys_1e9 > $R/$O/prof.log 2>&1 || exit 1
cut -d, -f1-4 $R/$O/prof/run_kernel_stats.csv | head -12
