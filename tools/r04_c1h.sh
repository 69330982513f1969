# C1 host-side check: the KEY_CACHING / batch tests, two C1 bench lines and
# the host sampler.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-c1h}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_chain_adapter.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/bench_c1_$r.json 2> $O/bench_c1_$r.err || { tail -20 $O/bench_c1_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['host'])" $O/bench_c1_$r.json
done
timeout -k 10 200 python tools/host_sample.py && mv gpurun_out/host_samples.txt gpurun_out/host_samples_libpsf.so $O/
