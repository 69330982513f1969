set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06l
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06l/gputest.log 2>&1
tail -2 gpurun_out/r06l/gputest.log
for c in c3 c3miss c1; do timeout -k 10 300 python bench.py --config $c --no-host-floor > gpurun_out/r06l/bench_$c.json 2> gpurun_out/r06l/bench_$c.err; tail -c 300 gpurun_out/r06l/bench_$c.json; echo; done
