set -e
mkdir -p gpurun_out/ab
for v in ${VARIANTS:-prev pre keep prevkeep prev pre keep prevkeep}; do
  PSF_LIBRARY_VARIANT=tools/variants/$v/libpsf.so timeout -k 10 120 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab/c4_$v.json 2>/dev/null
  python -c "
import json;d=json.load(open('gpurun_out/ab/c4_$v.json'));k=d['roofline']['kernels'];print('$v',d['value'],d['ms_per_step'],{a:b['avg_us'] for a,b in k.items()})"
done
