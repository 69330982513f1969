# A/B of single-array FIXING_FLOAT variants on the default bench (C2, 2^28):
# the parity tests, then `bench.py --no-cpu-baseline` per variant.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_c2}; shift; mkdir -p $O
for v in base "$@" base; do
  if [ $v = base ]; then L=""; else L=tools/variants/$v/libpsf.so; fi
  PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_$v.json 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], (d.get('config_128M') or {}).get('value'), {k:v['avg_us'] for k,v in d['roofline']['kernels'].items()})"
done
