cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
timeout -k 10 200 python tools/host_sample.py || exit 1
timeout -k 10 120 python tools/snappy_trace.py --run --mib 128 --kind codes || exit 1
timeout -k 10 120 python tools/snappy_trace.py --run --mib 128 --kind random || exit 1
