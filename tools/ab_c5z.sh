# same-box A/B of the C5 + COMPRESSING hit line: current build vs tools/variants/$V (default head),
# alternating, after the snappy / stored / fused tests with the current build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-abc5z}; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_stored.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2 3; do for v in cur ${V:-head}; do
  if [ $v = cur ]; then L=""; else L=$R/tools/variants/$v/libpsf.so; fi
  PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python bench.py --config c5 --compress --no-cpu-baseline > $O/b_${v}_$i.json 2>&1 || exit 1
  python3 -c "
import json
d=json.loads(open('$O/b_${v}_$i.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], {k:v['avg_us'] for k,v in d['roofline']['kernels'].items()})"
done; done
