cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
for c in c1 c3 c3miss; do
  timeout -k 10 300 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['host']; print(sys.argv[2], d['value'], d['ms_per_step'], d['steps'], 'active', h['active_ms_per_step'], 'blocked', h['blocked_ms_per_step'], 'kernel', h['kernel_ms_per_step'], (d.get('config_wire') or {}).get('value'), d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))" $O/bench_$c.json $c
done
