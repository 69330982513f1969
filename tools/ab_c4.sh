# A/B of libpsf variants (tools/build_variants.sh) on one bench config:
#   VARIANTS="a b" CONFIG=c4 bash tools/ab_c4.sh
set -e
mkdir -p gpurun_out/ab
CONFIG=${CONFIG:-c4}
for v in ${VARIANTS:-base}; do
  PSF_LIBRARY_VARIANT=tools/variants/$v/libpsf.so timeout -k 10 120 python bench.py --config $CONFIG --steps 20 --warmup 3 --no-cpu-baseline --no-128m > gpurun_out/ab/${CONFIG}_$v.json 2>/dev/null
  python -c "
import json;d=json.load(open('gpurun_out/ab/${CONFIG}_$v.json'));k=d['roofline']['kernels'];print('$v',d['value'],d['ms_per_step'],{a:b['avg_us'] for a,b in k.items()})"
done
