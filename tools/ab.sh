#!/bin/bash
# A/B runner for libpsf variants (tools/build_variants.sh builds them into
# tools/variants/<name>/libpsf.so; "base" = the in-tree libpsf.so).  Runs the
# bench configs for every variant, ROUNDS times in alternation (boxes drift;
# alternation keeps the comparison fair), one JSON line per run in
# gpurun_out/<label>/runs.jsonl, then prints per variant and config the
# median value and the per-kernel average times.
#
#   ROUNDS=3 CONFIGS="c2 c4 c5" EXTRA="--steps 20" tools/ab.sh <label> base v1 v2
#   TESTS="tests/test_gpu_batch.py" ...   (each variant runs these tests first)
#   ENVS="PSF_X=0 PSF_X=1" tools/ab.sh <label> base   (env A/B instead of libraries)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
label=$1; shift
O=gpurun_out/$label
mkdir -p $O
: > $O/runs.jsonl
ROUNDS=${ROUNDS:-2}
CONFIGS=${CONFIGS:-c2}
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=(base)
ENVLIST=(${ENVS:-""})
[ ${#ENVLIST[@]} -eq 0 ] && ENVLIST=("")
for v in "${VARIANTS[@]}"; do
  L=""; [ "$v" != base ] && L=tools/variants/$v/libpsf.so
  if [ -n "$TESTS" ]; then
    PSF_LIBRARY_VARIANT=$L timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread \
      > $O/tests_$v.log 2>&1 || { echo "tests failed for $v"; tail -30 $O/tests_$v.log; exit 1; }
  fi
done
for r in $(seq 1 $ROUNDS); do
  for v in "${VARIANTS[@]}"; do
    L=""; [ "$v" != base ] && L=tools/variants/$v/libpsf.so
    for e in "${ENVLIST[@]}"; do
      for c in $CONFIGS; do
        args="--config $c"
        case $c in c5z) args="--config c5 --compress";; c5zm) args="--config c5 --compress --miss";; esac
        out=$(env $e PSF_LIBRARY_VARIANT=$L timeout -k 10 300 python bench.py $args --no-cpu-baseline $EXTRA 2>$O/err.log | tail -1) \
          || { echo "bench failed: $v $e $c"; tail -20 $O/err.log; exit 1; }
        echo "{\"variant\": \"$v\", \"env\": \"$e\", \"config\": \"$c\", \"round\": $r, \"line\": $out}" >> $O/runs.jsonl
        echo "$r $v [$e] $c $(echo "$out" | grep -o '"value": [0-9.]*' | head -1)"
      done
    done
  done
done
python3 - "$O/runs.jsonl" <<'EOF'
import json, statistics, sys
from collections import defaultdict
runs = [json.loads(l) for l in open(sys.argv[1])]
g = defaultdict(list)
for r in runs:
    g[(r["config"], r["variant"], r["env"])].append(r["line"])
for (c, v, e), lines in sorted(g.items()):
    vals = [l["value"] for l in lines]
    ks = defaultdict(list)
    for l in lines:
        for k, d in ((l.get("roofline") or {}).get("kernels") or {}).items():
            ks[k].append(d["avg_us"])
    print(f"{c:5s} {v:12s} {e:24s} value median {statistics.median(vals):9.1f} {vals} ",
          {k: round(statistics.median(x), 1) for k, x in ks.items()})
EOF
