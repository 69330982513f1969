#!/bin/bash
# A/B of snappy variants (tools/build_variants.sh with SRC=.../snappy.hip) on
# bench_snappy payloads: `tools/gpu_snappy_ab.sh <out> <payloads> <variant|base>...`
# (set TESTS=1 to run the snappy GPU tests on the in-tree build first;
# ABFLAGS=--no-verify to time the uncompress as well).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; O=gpurun_out/$1; P=$2; shift 2; mkdir -p $O; export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_bounded.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for v in "$@"; do
  if [ "$v" = base ]; then unset PSF_LIBRARY_VARIANT; else export PSF_LIBRARY_VARIANT=tools/variants/$v/libpsf.so; fi
  echo "== $v"
  timeout -k 10 200 python3 tools/bench_snappy.py --mib 128 --no-cpu ${ABFLAGS:---no-check} --reps ${REPS:-2} --only $P > $O/b_$v.log 2>&1 || exit 1
  grep payload $O/b_$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['payload'], d['ratio'], 'compress', d.get('snappy_compress_kernel_ms'), 'ms; uncompress', d.get('snappy_decompress_kernel_ms'), 'ms')"
done
