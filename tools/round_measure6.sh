#!/bin/bash
# Round-6 measurement session for profiles/: the GPU test suite, smoke(), every
# bench line (the default command as the driver runs it, then C1 / C3 / C3miss
# / C4 / C4pull / C5 / C5+COMPRESSING hit and miss), snappy alone, the host
# edge, rocprofv3 kernel-trace stats of every line and PMC passes of every
# line (FETCH_SIZE, WRITE_SIZE, each its own run, --pmc only).  Every GPU step
# has its own time limit and the session stops at the first failure.
# Output: gpurun_out/$TAG/.  tools/save_profiles6.sh copies it to profiles/.
#   STEPS="tests bench prof pmc" /usr/local/graft/bin/gpurun -- 'bash tools/round_measure6.sh r06z'
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r06z}
O=gpurun_out/$TAG
mkdir -p $O
set -o pipefail
R=$PWD
S=" ${STEPS:-tests bench prof pmc} "
if [[ $S == *" tests "* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
  tail -2 $O/gputest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [[ $S == *" bench "* ]]; then
  timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('config_128M') or {}).get('value'), (d.get('config_c4') or {}).get('value'), d['cpu_baseline'])"
  for c in "c1" "c3" "c3miss" "c4" "c4pull" "c5" "c5 --compress" "c5 --compress --miss"; do
    n=$(echo $c | tr -d ' -' )
    timeout -k 10 300 python bench.py --config $c > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/bench_$n.json')); print('$n', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel'), (d.get('roofline') or {}).get('frac'))"
  done
  timeout -k 10 300 python -u tools/bench_snappy.py --mib 128 > $O/bench_snappy.jsonl 2> $O/bench_snappy.err || exit 1
  timeout -k 10 300 python -u tools/host_edge_chain.py --out $O/host_edge.jsonl > $O/host_edge.log 2>&1 || exit 1
fi
cd /tmp
LINES=("c2:--no-128m --no-c4" "c1:--config c1" "c3:--config c3" "c4:--config c4" "c4pull:--config c4pull"
       "c5:--config c5" "c5z:--config c5 --compress")
if [[ $S == *" prof "* ]]; then
  for cfg in "${LINES[@]}"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$name -o run -- \
      python3 $R/bench.py $args --no-cpu-baseline --no-host-floor > $R/$O/prof_$name.log 2>&1 || { tail -20 $R/$O/prof_$name.log; exit 1; }
  done
fi
if [[ $S == *" pmc "* ]]; then
  for cfg in "${LINES[@]}"; do
    name=${cfg%%:*}; args=${cfg#*:}
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_${name}_fetch -o run -- python3 $R/bench.py $args --no-cpu-baseline --no-profile --no-host-floor --steps 5 --warmup 1 > $R/$O/pmc_${name}_fetch.log 2>&1 || exit 1
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_${name}_write -o run -- python3 $R/bench.py $args --no-cpu-baseline --no-profile --no-host-floor --steps 5 --warmup 1 > $R/$O/pmc_${name}_write.log 2>&1 || exit 1
  done
fi
echo done
