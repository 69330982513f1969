# A/B of the parallel window linker (K2p, PSF_LINK_PARALLEL, default on):
# the snappy / fused / stored tests, then 128 MiB sorted keys both ways and a
# kernel-trace of the default.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-link}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_snappy.py tests/test_gpu_fused.py tests/test_gpu_bounded.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for f in 1 0 1 0; do
  echo "PSF_LINK_PARALLEL=$f"
  PSF_LINK_PARALLEL=$f timeout -k 10 200 python -u tools/bench_snappy.py --mib 128 --no-cpu --only sorted_keys_1e9 2>&1 | grep payload || exit 1
done
R=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/tools/bench_snappy.py --mib 128 --no-cpu --only sorted_keys_1e9 > $R/$O/prof.log 2>&1 || exit 1
cut -d, -f1-4 $R/$O/prof/run_kernel_stats.csv | head -12
