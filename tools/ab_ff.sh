# A/B of batched FIXING_FLOAT grid variants (tools/build_variants.sh builds of
# ff_codec.hip): the batch tests, then bench C5 and C4 per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_ff}; shift; mkdir -p $O
for v in base "$@" base; do
  if [ $v = base ]; then L=""; else L=tools/variants/$v/libpsf.so; fi
  PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python -m pytest tests/test_gpu_batch.py -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  for c in c5 c4; do
    PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_$v.json 2>&1 || exit 1
  done
  echo $v c5 $(grep -o '"value": [0-9.]*' $O/b_c5_$v.json | head -1) c4 $(grep -o '"value": [0-9.]*' $O/b_c4_$v.json | head -1)
  python3 -c "
import json,sys
for c in ('c5','c4'):
    d=json.loads(open('$O/b_'+c+'_$v.json').read().strip().splitlines()[-1])
    print('  ',c,{k:v['avg_us'] for k,v in d['roofline']['kernels'].items()})"
done
