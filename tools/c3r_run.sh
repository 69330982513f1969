# tools/c3real_probe builds under rocprofv3 (one GPU call), then the traced build:
#   bash tools/c3r_run.sh "<probe args>" bin1 bin2 ...
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c3r; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A=$1; shift
for b in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$b -o run -- $R/tools/$b 300 $A >> $O/log.txt 2>&1
done
if [ -x $R/tools/c3real_probe_tr ]; then timeout -k 10 60 $R/tools/c3real_probe_tr 300 $A > $O/trace.txt 2>&1; fi
if [ -x $R/tools/c3real_probe_trnpf ]; then timeout -k 10 60 $R/tools/c3real_probe_trnpf 300 $A > $O/trace_npf.txt 2>&1; fi
