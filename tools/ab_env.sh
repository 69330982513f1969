#!/bin/bash
# A/B of run-time knobs on the default bench (C2, 2^28): the parity tests once,
# then bench.py per setting; each argument is one setting, a space-separated
# list of VAR=value assignments ("-" for none), e.g.
#   tools/ab_env.sh ab1 PSF_FF_REORDER=0 PSF_FF_REORDER=1 "PSF_FF_REORDER=1 PSF_FF_KEEP_MIB=64"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_env}; shift; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
i=0
for setting in "$@"; do
  i=$((i+1))
  envs=(); [ "$setting" = "-" ] || read -ra envs <<< "$setting"
  env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_$i.json 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_$i.json').read().strip().splitlines()[-1])
print('$setting', d['value'], d['ms_per_step'], (d.get('config_128M') or {}).get('value'), {k:v['avg_us'] for k,v in d['roofline']['kernels'].items()})"
done
