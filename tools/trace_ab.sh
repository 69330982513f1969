cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in trace_base trace_lds; do for k in codes random; do
  timeout -k 10 120 python tools/snappy_trace.py --run --name $v --kind $k --mib 128 >> gpurun_out/trace.log 2>&1 || exit $?
done; timeout -k 10 120 python tools/snappy_trace.py --run --name $v --kind keys --mib 32 >> gpurun_out/trace.log 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/trace.log
