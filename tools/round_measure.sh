#!/bin/bash
# One measurement session for profiles/: the GPU test suite, the bench lines
# (default C2 and the C1 / C4 / C5 / C5+COMPRESSING configs, CPU baselines
# included), rocprofv3 kernel-trace stats of C2 and C4, and the C4 PMC passes
# (FETCH_SIZE, WRITE_SIZE, each its own run).  Output: gpurun_out/$TAG/.
#   /usr/local/graft/bin/gpurun -- 'bash tools/round_measure.sh r02c'
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${1:-r02c}
O=gpurun_out/$TAG
mkdir -p $O
set -o pipefail
R=$PWD
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
for c in c1 c4 c5; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
done
timeout -k 10 300 python bench.py --config c5 --compress > $O/bench_c5_compress.json 2> $O/bench_c5_compress.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/prof_c2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c4 -o run -- python3 $R/bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/prof_c4.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_c5z -o run -- python3 $R/bench.py --config c5 --compress --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/prof_c5z.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_c4_fetch -o run -- python3 $R/bench.py --config c4 --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $R/$O/pmc_c4_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_c4_write -o run -- python3 $R/bench.py --config c4 --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $R/$O/pmc_c4_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_c5z_fetch -o run -- python3 $R/bench.py --config c5 --compress --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $R/$O/pmc_c5z_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_c5z_write -o run -- python3 $R/bench.py --config c5 --compress --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $R/$O/pmc_c5z_write.log 2>&1 || exit $?
cd $R
if [ -f tools/variants/hprof/libpsf.so ]; then
  timeout -k 10 150 python tools/host_prof.py > $O/hprof_c1.txt 2>&1 || exit $?
fi
echo done
