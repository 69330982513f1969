#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault-like exit (timeout, abort,
# segfault, kill) ends the script at once.  Test failures (exit 1) do not.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fault-like exit from $name; stopping"; exit $rc
  fi
  return 0
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    pytestall) step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread ;;
    hostedge) step host_edge 300 python tools/host_edge.py ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    benchq) step bench 600 python bench.py --no-cpu-baseline --steps 20 ;;
    prof) step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 20 ;;
    *) echo "unknown step $s" ;;
  esac
done
