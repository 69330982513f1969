set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_check.sh pytest smoke bench || exit $?
timeout -k 10 600 python tools/host_edge_chain.py > gpurun_out/host_edge_chain.log 2>&1; echo "host_edge rc=$?"; tail -8 gpurun_out/host_edge_chain.log
