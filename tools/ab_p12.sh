# A/B of the 12-wave compress parse workgroups against the 8-wave build
# (tools/variants/p8): snappy / stored / timed-size tests, then C5 +
# COMPRESSING hit and miss lines both ways.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-p12}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_stored.py tests/test_gpu_timed_sizes.py tests/test_gpu_bounded.py -x -q \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for v in cur p8; do
    if [ $v = cur ]; then unset PSF_LIBRARY_VARIANT; else export PSF_LIBRARY_VARIANT=tools/variants/p8/libpsf.so; fi
    for c in "--config c5 --compress" "--config c5 --compress --miss"; do
      f=$O/b_${v}_$(echo $c | tr -d ' -')_$r.json
      timeout -k 10 300 python bench.py $c --no-cpu-baseline > $f 2> $f.err || { tail -30 $f.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['roofline']['kernels'].items()})" $f "$v $c"
    done
  done
done
unset PSF_LIBRARY_VARIANT
timeout -k 10 200 python -u tools/bench_snappy.py --mib 128 --no-cpu 2>&1 | grep payload
