# GPU check of a snappy parse change: the snappy / stored / bounded tests,
# then the compress benchmark over all payloads and C5 + COMPRESSING.
# Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-win}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_stored.py tests/test_gpu_bounded.py \
  -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/bench_snappy.py --mib 128 --no-cpu > $O/bench_snappy.txt 2>&1 || { tail -30 $O/bench_snappy.txt; exit 1; }
cat $O/bench_snappy.txt
for c in "--config c5 --compress" "--config c5 --compress --miss"; do
  f=$O/bench_$(echo $c | tr -d ' -').json
  timeout -k 10 300 python bench.py $c --no-cpu-baseline > $f 2> $f.err || { tail -30 $f.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['roofline']['kernels'].items()})" $f "$c"
done
