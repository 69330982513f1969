# kernel stats of C5 + COMPRESSING (hits), rocprofv3 kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-prof_c5z}; mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O -o run -- python3 $R/bench.py --config c5 --compress ${2:-} --no-cpu-baseline --steps 20 --warmup 3 > $R/$O/bench.log 2>&1 || exit 1
find $R/$O -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | sed 's/(psf::[^"]*//' | head -14
