# Quick GPU check after a codec change: the stored-layout, C4/C5 timed-size,
# fused, snappy and spill tests, then C5 (+ COMPRESSING, hits / misses) bench
# lines.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_stored.py tests/test_gpu_timed_sizes.py tests/test_gpu_fused.py \
  tests/test_gpu_snappy.py tests/test_gpu_spill.py -x -v --timeout 240 --timeout-method thread > $O/quick.log 2>&1 \
  || { tail -60 $O/quick.log; exit 1; }
tail -2 $O/quick.log
for c in "--config c5" "--config c5 --compress" "--config c5 --compress --miss"; do
  f=$O/bench_$(echo $c | tr -d ' -').json
  timeout -k 10 300 python bench.py $c --no-cpu-baseline > $f 2> $f.err || { tail -30 $f.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['roofline']['kernels'].items()})" $f "$c"
done
