# A/B of router-step variants (C5 + COMPRESSING, C5, C4) on one box:
# base and the given tools/variants builds, alternated.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_router}; shift; mkdir -p $O
for v in base "$@" base "$@"; do
  if [ $v = base ]; then L=""; else L=tools/variants/$v/libpsf.so; fi
  for c in "c5 --compress" c5 c4; do
    PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python bench.py --config $c --no-cpu-baseline 2>/dev/null | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);h=d['host'];print('$v','$c',d['value'],d['ms_per_step'],h['active_ms_per_step'],h['kernel_ms_per_step'])" || exit 1
  done
done
