#!/bin/bash
# Copy one tools/round_measure6.sh session (gpurun_out/<tag>/) into
# profiles/<tag>/: bench lines, rocprofv3 kernel stats of every line, the PMC
# traffic of every line (also profiles/pmc_traffic.json, which bench.py reads
# for roofline.traffic), snappy / host-edge lines, the GPU suite's tail.
#   tools/save_profiles6.sh r06z
set -e
cd "$(dirname "$0")/.."
T=$1; O=gpurun_out/$T; P=profiles/$T
mkdir -p $P
python tools/pmc_traffic.py $O --out profiles/pmc_traffic.json
cp profiles/pmc_traffic.json $P/pmc_traffic.json
for c in c2 c1 c3 c4 c4pull c5 c5z; do
  f=$(find $O/prof_$c -name "*kernel_stats.csv" | head -1)
  [ -n "$f" ] && cp $f $P/${c}_kernel_stats.csv
  fd=$O/pmc_${c}_fetch; wd=$O/pmc_${c}_write
  [ -d $fd ] && python tools/pmc_summary.py $fd $wd --only psf:: --json $P/pmc_$c.json > /dev/null
done
for c in default c1 c3 c3miss c4 c4pull c5 c5compress c5compressmiss; do cp $O/bench_$c.json $P/bench_$c.json; done
cp $O/bench_snappy.jsonl $P/bench_snappy.jsonl
cp $O/host_edge.jsonl $P/host_edge_chain.jsonl
(tail -2 $O/gputest.log; tail -1 $O/smoke.log) > $P/gputest_tail.txt
echo saved $T
