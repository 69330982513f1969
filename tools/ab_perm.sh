# A/B of the encode's workgroup order after the min/max pass (PSF_ENC_PERM,
# default on) on the default bench (C2, 2^28): parity tests, then bench.py
# --no-cpu-baseline alternating off / on, three times.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_perm}; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2 3; do for v in 0 1; do
  PSF_ENC_PERM=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_${v}_${i}.json 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_${v}_${i}.json').read().strip().splitlines()[-1])
print('perm=$v', d['value'], d['ms_per_step'], (d.get('config_128M') or {}).get('value'), {k:v['avg_us'] for k,v in d['roofline']['kernels'].items()})"
done; done
