# tag-dense uncompress A/B: the snappy / fused / bounded tests with the
# current build (or tools/variants/$TESTVAR), then tools/bench_snappy.py (sorted keys, zeros) with each of
# tools/variants/$VARS twice, and a kernel trace of each.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-abdec}; mkdir -p $O
${TESTVAR:+env PSF_LIBRARY_VARIANT=$R/tools/variants/$TESTVAR/libpsf.so} timeout -k 10 500 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_fused.py tests/test_gpu_bounded.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in $VARS; do
  echo "== $v"
  PSF_LIBRARY_VARIANT=$R/tools/variants/$v/libpsf.so timeout -k 10 200 python -u tools/bench_snappy.py --mib 128 --no-cpu --only ${ONLY:-sorted_keys_1e9,zeros} 2>&1 | grep payload | cut -c1-170 || exit 1
done
done
for v in $VARS; do
  (cd /tmp && PSF_LIBRARY_VARIANT=$R/tools/variants/$v/libpsf.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o run -- python3 $R/tools/bench_snappy.py --mib 128 --no-cpu --only sorted_keys_1e9 > $R/$O/$v.log 2>&1) || exit 1
  echo "== $v kernels"
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if 'snappy' in n: print(n[n.index('snappy'):].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms')
" $O/$v/run_kernel_stats.csv
done
