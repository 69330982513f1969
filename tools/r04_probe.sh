# the snappy probe's fast path: GPU snappy tests, the probe trace, C5z bench + kernel stats
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py -x -q --timeout 120 --timeout-method thread > $O/test.txt 2>&1 || { tail -30 $O/test.txt; exit 1; }
tail -2 $O/test.txt
timeout -k 10 120 python -u tools/snappy_trace.py --run --mib 128 --kind codes > $O/tr_codes.txt 2>&1 || exit 1
tail -1 $O/tr_codes.txt
timeout -k 10 300 python bench.py --config c5 --compress --no-cpu-baseline > $O/bench_c5z.json 2> $O/bench_c5z.err || { tail -20 $O/bench_c5z.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5z', d['value'], d['ms_per_step'])" $O/bench_c5z.json
bash tools/prof_c5z_quick.sh r04p/prof_c5z
