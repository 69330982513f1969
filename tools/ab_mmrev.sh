# A/B: the batched min/max pass dispatched last-array-first (PSF_MM_REVERSE=1)
# so the encode's first arrays come from the Infinity Cache; C5 and C5 +
# COMPRESSING, alternating.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-ab_mmrev}; mkdir -p $O
for rep in 1 2; do
  for r in 0 1; do
    for z in "" "--compress"; do
      PSF_MM_REVERSE=$r timeout -k 10 200 python bench.py --config c5 $z --no-cpu-baseline --steps 30 > $O/c5_${r}${z}_$rep.json 2>/dev/null || exit 1
      python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(sys.argv[1], d['value'], d['ms_per_step'], k.get('ff_minmax_partials',{}).get('avg_us'), k.get('ff_encode',{}).get('avg_us'))" $O/c5_${r}${z}_$rep.json
    done
  done
done
