# same-box A/B of the router's prefetched slicing on the side stream
# (PSF_SIDE_SLICE, default on): the router / timed-size tests, then C4, C5 and
# C5 + COMPRESSING alternating off / on
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_side_slice}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_sizes.py tests/test_gpu_spill.py tests/test_gpu_consumer.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do for c in "c4" "c5" "c5 --compress"; do for v in 0 1; do
  n=$(echo $c | tr -d ' -')
  PSF_SIDE_SLICE=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $O/b_${n}_${v}_$i.json 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_${n}_${v}_$i.json').read().strip().splitlines()[-1])
h=d['host']
print('$n side=$v', d['value'], d['ms_per_step'], 'active', round(h['active_ms_per_step'],4), 'blocked', round(h['blocked_ms_per_step'],4), 'kernel', h['kernel_ms_per_step'])"
done; done; done
