# kernel stats of the stored-payload uncompress, current build vs tools/variants/old
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-ringprof}; mkdir -p $O
for v in new old; do
  if [ $v = old ]; then export PSF_LIBRARY_VARIANT=$R/tools/variants/old/libpsf.so; else unset PSF_LIBRARY_VARIANT; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/$v -o run -- python3 $R/tools/bench_snappy.py --mib 128 --no-cpu --only ff_codes_nb1,random --reps 10 > $R/$O/$v.log 2>&1) || exit 1
  echo "== $v"; grep payload $O/$v.log
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'snappy' in r['Name']: print(r['Name'].split('(')[1].split('::')[-1] if '::' in r['Name'] else r['Name'], r['Calls'], r['AverageNs'])
" $O/$v/run_kernel_stats.csv
done
