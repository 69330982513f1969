# fragment-decoder ablation (diagnostic): kernel averages of sorted-key
# uncompress with tools/variants/{cur,nocopy,nolit} (no verification)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-abdfrag}; mkdir -p $O
for v in ${VARS:-cur nocopy nolit}; do
  (cd /tmp && PSF_LIBRARY_VARIANT=$R/tools/variants/$v/libpsf.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o run -- python3 $R/tools/bench_snappy.py --mib 128 --no-cpu --no-verify --only sorted_keys_1e9 > $R/$O/$v.log 2>&1) || exit 1
  echo "== $v"
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if 'snappy_d' in n: print(n[n.index('snappy'):].split('(')[0], r['Calls'], round(float(r['AverageNs'])/1e6,3), 'ms')
" $O/$v/run_kernel_stats.csv
done
