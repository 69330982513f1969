# A/B of the decode tiles per workgroup inside ff_fused_batch (C1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ftpw}; mkdir -p $O
for r in 1 2; do
  for t in 4 8 16; do
    PSF_FUSED_DEC_TPW=$t timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline > $O/c1_t${t}_$r.json 2> $O/c1_t${t}_$r.err || { tail -20 $O/c1_t${t}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['host']; print(sys.argv[2], d['value'], d['ms_per_step'], 'active', h['active_ms_per_step'], 'kernel', h['kernel_ms_per_step'], {k: (v['launches'], v['avg_us']) for k, v in d['roofline']['kernels'].items()})" $O/c1_t${t}_$r.json "tpw=$t"
  done
done
