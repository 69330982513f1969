# PMC passes over the tag-dense snappy kernels (128 MiB of sorted keys, one
# compress + uncompress): instruction mix and stall cycles (two SQ passes) and
# HBM traffic (FETCH_SIZE, WRITE_SIZE), each counter set its own run, nothing
# but --pmc (no tracing domain).  Summary: tools/pmc_sq_summary.py.
# Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-pmc_sorted}; mkdir -p $O
cd /tmp
CMD="python3 $R/tools/bench_snappy.py --mib 128 --only sorted_keys_1e9 --no-cpu --reps 1"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- $CMD > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python3 $R/tools/pmc_sq_summary.py $O
