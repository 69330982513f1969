# A/B of the stored-layout encode: probe sheet on / off (PSF_STORED_SHEET),
# C5 + COMPRESSING; then one rocprofv3 kernel-trace of each for the split of
# the compressor's launches.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_stored}; mkdir -p $O
for rep in 1 2; do
  for sh in 1 0; do
    PSF_STORED_SHEET=$sh timeout -k 10 200 python bench.py --config c5 --compress --no-cpu-baseline --steps 30 > $O/c5z_sheet${sh}_$rep.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(sys.argv[1], d['value'], d['ms_per_step'], {n: v['avg_us'] for n, v in k.items()})" $O/c5z_sheet${sh}_$rep.json
  done
done
for sh in 1 0; do
  PSF_STORED_SHEET=$sh timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_sheet$sh -o run -- python bench.py --config c5 --compress --no-cpu-baseline --no-profile --steps 20 > /dev/null 2>&1 || exit 1
  f=$(find $O/prof_sheet$sh -name "*kernel_stats.csv" | head -1); echo "== sheet $sh"; cut -d, -f1-4 $f | head -12
done
