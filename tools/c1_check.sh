# C1 (ctr triple x 64 streams): the bench line (with config_wire) and the
# host-section profile (diagnostic build tools/variants/hprof).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-c1}; mkdir -p $O
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || { tail -20 $O/bench_c1.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('c1', d['value'], d['ms_per_step'], d['host'], d.get('config_wire')); print({k: (v['launches'], v['avg_us']) for k, v in d['roofline']['kernels'].items()})" $O/bench_c1.json
if [ -f tools/variants/hprof/libpsf.so ]; then
  timeout -k 10 200 python tools/host_prof.py > $O/hprof_c1.txt 2>&1 || exit 1
  cat $O/hprof_c1.txt
fi
