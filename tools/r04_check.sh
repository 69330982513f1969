# Round 4 GPU check: the whole -m gpu suite, then the default bench line and
# C5 + COMPRESSING (hits and misses).  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r04}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > $O/gputest.log 2>&1 || { tail -60 $O/gputest.log; exit 1; }
tail -3 $O/gputest.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
for m in "" "--miss"; do
  timeout -k 10 300 python bench.py --config c5 --compress $m --no-cpu-baseline > $O/bench_c5z$m.json 2> $O/bench_c5z$m.err \
    || { tail -30 $O/bench_c5z$m.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['roofline']['kernels'].items()})" $O/bench_c5z$m.json
done
