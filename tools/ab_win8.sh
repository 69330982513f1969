# window size A/B for the tag-dense uncompress (K1-K3): tools/variants/{cur,w8}
# (16 and 8 KiB windows): the snappy / fused tests with w8, then
# tools/bench_snappy.py on sorted keys and zeros, twice each, and kernel traces.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-win8}; mkdir -p $O
PSF_LIBRARY_VARIANT=$R/tools/variants/w8/libpsf.so timeout -k 10 500 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_fused.py tests/test_gpu_bounded.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for v in ${VARS:-cur w8}; do
  echo "== $v"
  PSF_LIBRARY_VARIANT=$R/tools/variants/$v/libpsf.so timeout -k 10 200 python -u tools/bench_snappy.py --mib 128 --no-cpu --only sorted_keys_1e9,zeros 2>&1 | grep payload | cut -c1-170 || exit 1
done
done
for v in ${VARS:-cur w8}; do
  (cd /tmp && PSF_LIBRARY_VARIANT=$R/tools/variants/$v/libpsf.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o run -- python3 $R/tools/bench_snappy.py --mib 128 --no-cpu --only sorted_keys_1e9 > $R/$O/$v.log 2>&1) || exit 1
  echo "== $v kernels"
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'snappy' in r['Name']: print(r['Name'].split('(')[0].split('::')[-1], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms')
" $O/$v/run_kernel_stats.csv
done
