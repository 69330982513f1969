# same-box A/B of PSF_ENC_PERM on the small-array configs (C1, C3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_perm_c13}; mkdir -p $O
for i in 1 2; do for c in c3 c1; do for v in 0 1; do
  PSF_ENC_PERM=$v timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/b_${c}_${v}_${i}.json 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_${c}_${v}_${i}.json').read().strip().splitlines()[-1])
print('$c perm=$v', d['value'], d['ms_per_step'], d['host']['active_ms_per_step'], d['host']['kernel_ms_per_step'], {k:v['avg_us'] for k,v in d['roofline']['kernels'].items()})"
done; done; done
