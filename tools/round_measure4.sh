#!/bin/bash
# Round-4 measurement session for profiles/: the GPU test suite, the bench
# lines (default C2 and C1 / C3 / C3miss / C4 / C5 / C5+COMPRESSING hit and
# miss, CPU baselines included), rocprofv3 kernel-trace stats of C2 at 2^28
# alone (--no-128m: one size per row) and of C5+COMPRESSING, and PMC passes
# (FETCH_SIZE, WRITE_SIZE, each its own run).  Output: gpurun_out/$TAG/.
#   STEPS="tests bench prof pmc" /usr/local/graft/bin/gpurun -- 'bash tools/round_measure4.sh r04z'
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r04z}
O=gpurun_out/$TAG
mkdir -p $O
set -o pipefail
R=$PWD
S=" ${STEPS:-tests bench prof pmc} "
if [[ $S == *" tests "* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || exit $?
  tail -3 $O/gputest.log
fi
if [[ $S == *" bench "* ]]; then
  timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
  for c in "c1" "c3" "c3miss" "c4" "c5" "c5 --compress" "c5 --compress --miss"; do
    n=$(echo $c | tr -d ' -' )
    timeout -k 10 300 python bench.py --config $c > $O/bench_$n.json 2> $O/bench_$n.err || exit $?
    python -c "import json,sys; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel'), (d.get('roofline') or {}).get('frac'), d.get('host'))"
  done
  timeout -k 10 300 python -u tools/bench_snappy.py --mib 128 > $O/bench_snappy.jsonl 2> $O/bench_snappy.err || exit $?
fi
cd /tmp
if [[ $S == *" prof "* ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c2 -o run -- python3 $R/bench.py --no-128m --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/prof_c2.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c5z -o run -- python3 $R/bench.py --config c5 --compress --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/prof_c5z.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c1 -o run -- python3 $R/bench.py --config c1 --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/prof_c1.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c4 -o run -- python3 $R/bench.py --config c4 --no-cpu-baseline --steps 10 --warmup 2 > $R/$O/prof_c4.log 2>&1 || exit $?
fi
if [[ $S == *" pmc "* ]]; then
  for cfg in "c2:--no-128m" "c5z:--config c5 --compress"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_${name}_fetch -o run -- python3 $R/bench.py $args --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $R/$O/pmc_${name}_fetch.log 2>&1 || exit $?
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_${name}_write -o run -- python3 $R/bench.py $args --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $R/$O/pmc_${name}_write.log 2>&1 || exit $?
  done
fi
echo done
