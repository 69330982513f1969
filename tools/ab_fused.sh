# A/B of ff_fused_batch (a small batch's min/max + encode + pending decode in
# one launch, the default) against two launches (PSF_FF_FUSED=0):
# the batched / parity / adapter tests with it on, then C1 and C3 lines both
# ways.  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-fused}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_parity.py tests/test_gpu_chain_adapter.py \
  tests/test_gpu_adapter.py tests/test_gpu_stored.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
  for f in 1; do
    for c in c1; do
      PSF_FF_FUSED=$f timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_${c}_f${f}_$r.json 2> $O/bench_${c}_f${f}_$r.err \
        || { tail -20 $O/bench_${c}_f${f}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['host']; print(sys.argv[2], d['value'], d['ms_per_step'], 'active', h['active_ms_per_step'], 'kernel', h['kernel_ms_per_step'], {k: (v['launches'], v['avg_us']) for k, v in d['roofline']['kernels'].items()})" $O/bench_${c}_f${f}_$r.json "$c fused=$f"
    done
  done
done
