#!/bin/bash
mkdir -p gpurun_out/r05e
for r in 1 2; do
  for v in "0 1024" "160 256" "160 512" "160 128"; do
    set -- $v
    PSF_FF_GROUP_MB=$1 PSF_FF_GROUP_MMWG=$2 timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > gpurun_out/r05e/b.json 2>gpurun_out/r05e/b.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/r05e/b.json')); k=d['roofline']['kernels']; print('$v', d['value'], {a: (v['launches'], v['avg_us']) for a, v in k.items()})"
  done
done
