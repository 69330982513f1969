# full GPU suite + smoke + default bench + C5 lines (hits, misses)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-full2}; mkdir -p $O
bash tools/r04_full.sh $1 || exit 1
timeout -k 10 300 python bench.py --config c5 --compress --no-cpu-baseline > $O/bench_c5z.json 2> $O/bench_c5z.err || { tail -20 $O/bench_c5z.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --compress --miss --no-cpu-baseline > $O/bench_c5z_miss.json 2> $O/bench_c5z_miss.err || { tail -20 $O/bench_c5z_miss.err; exit 1; }
for f in c5z c5z_miss; do python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(sys.argv[2], d['value'], d['ms_per_step'], {n: v['avg_us'] for n, v in k.items()})" $O/bench_$f.json $f; done
