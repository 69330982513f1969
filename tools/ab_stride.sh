#!/bin/bash
# What the live timing of the dominant kernel costs each line: stride 1 / 4 /
# no live timing, alternated.   tools/ab_stride.sh <label>
O=gpurun_out/${1:-ab_stride}; mkdir -p $O
for r in 1 2 3; do
  for c in "c2 --no-128m --no-c4" "c3" "c5" "c5 --compress"; do
    for v in "--prof-stride 1" "--prof-stride 4" "--no-profile"; do
      timeout -k 10 300 python bench.py --config $c --no-cpu-baseline $v > $O/b.json 2> $O/b.err || exit 1
      python -c "import json; d=json.load(open('$O/b.json')); print('$c', '$v', d['value'], (d.get('roofline') or {}).get('avg_us'), (d.get('roofline') or {}).get('launches_timed'))"
    done
  done
done
