#!/bin/bash
# A/B of snappy variants (tools/snappy_variant.sh builds) on one payload: kernel stats per variant
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=${P:-ff_codes_nb1}
for v in "$@"; do
  if [ "$v" = base ]; then unset PSF_LIBRARY_VARIANT; else export PSF_LIBRARY_VARIANT=tools/variants/$v/libpsf.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python3 tools/bench_snappy.py --mib 128 --no-cpu --only $P > gpurun_out/ab_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/ab_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -v amdgpu.ids gpurun_out/ab_$v.log | tail -1; grep "snappy" "$f" | cut -d, -f1-4 | sed 's/psf::(anonymous namespace):://; s/(psf[^"]*"/"/'
done
