# snappy compress of sorted keys at several sizes (per-fragment parse rates
# of the staged and the from-memory paths)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for m in 16 32 64 128; do
  timeout -k 10 120 python -u tools/bench_snappy.py --mib $m --no-cpu --only sorted_keys_1e9 2>&1 | grep payload || exit 1
done
