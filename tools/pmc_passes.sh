#!/bin/bash
# rocprofv3 PMC passes over bench configurations: two SQ passes (wave states
# and the instruction mix), then FETCH_SIZE and WRITE_SIZE -- each counter set
# its own run, --pmc only (no tracing domain), each under its own time limit.
# Per-kernel sums: tools/pmc_sq_summary.py, written to <out>/<name>.json.
#   bash tools/pmc_passes.sh <label> "c2:--no-128m --no-c4" "c3:--config c3" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/${1:-pmc}; shift
mkdir -p $O
cd /tmp
for cfg in "$@"; do
  name=${cfg%%:*}; args=${cfg#*:}
  mkdir -p $O/$name
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
             "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $O/$name/p$i -o run -- \
      python3 $R/bench.py $args --no-cpu-baseline --no-profile --steps 5 --warmup 1 > $O/$name/p$i.log 2>&1 \
      || { echo "$name pass $i failed"; tail -5 $O/$name/p$i.log; exit 1; }
  done
  python3 $R/tools/pmc_sq_summary.py $O/$name --json $O/$name.json > /dev/null
  echo "$name done"
done
