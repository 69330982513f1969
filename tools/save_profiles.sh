#!/bin/bash
# Copy one tools/round_measure5.sh session (gpurun_out/<tag>/) into profiles/<tag>_*:
# bench lines, rocprofv3 kernel stats, PMC summaries, snappy / host-edge lines,
# the GPU suite's tail.   tools/save_profiles.sh r05w
set -e
cd "$(dirname "$0")/.."
T=$1; O=gpurun_out/$T; P=profiles
for c in c2 c5z; do
  f=$(find $O/pmc_${c}_fetch -name "*counter_collection.csv" | head -1); w=$(find $O/pmc_${c}_write -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $(dirname $f) $(dirname $w) --only psf:: --json $P/${T}_pmc_$c.json > /dev/null
  [ $c = c2 ] && python tools/pmc_traffic.py --fetch $f --write $w --n 268435456 --nb 1 --out $P/pmc_traffic.json > /dev/null
done
for c in c1 c2 c4 c5z; do cp $(find $O/prof_$c -name "*kernel_stats.csv" | head -1) $P/${T}_${c}_kernel_stats.csv; done
for c in c1 c3 c3miss c4 c5 c5compress c5compressmiss default; do cp $O/bench_$c.json $P/${T}_bench_$c.json; done
cp $O/bench_snappy.jsonl $P/${T}_bench_snappy.jsonl
cp $O/host_edge.jsonl $P/${T}_host_edge_chain.jsonl
(tail -2 $O/gputest.log; tail -1 $O/smoke.log) > $P/${T}_gputest_tail.txt
echo saved $T
