# A/B of the fused dequantise's load variants (tools/build_variants.sh builds):
# each variant's fused-decode tests, then bench --config c5 --compress.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab_dq}; shift; mkdir -p $O
for v in base "$@" base; do
  if [ $v = base ]; then L=""; else L=tools/variants/$v/libpsf.so; fi
  PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1 || { tail -20 $O/t_$v.log; exit 1; }
  PSF_LIBRARY_VARIANT=$L timeout -k 10 200 python bench.py --config c5 --compress --no-cpu-baseline > $O/b_$v.json 2>&1 || exit 1
  echo $v $(grep -o '"value": [0-9.]*' $O/b_$v.json | head -1) $(grep -o '"kernel": "snappy_decompress", "avg_us": [0-9.]*' $O/b_$v.json)
done
