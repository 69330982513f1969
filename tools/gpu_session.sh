set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r; mkdir -p $O
TESTS="tests/test_gpu_snappy.py tests/test_gpu_stored.py" ROUNDS=3 CONFIGS="c5z c5zm" EXTRA="--no-host-floor" timeout -k 10 1000 bash tools/ab.sh r06r_place base pt512 pt1024 > $O/ab.log 2>&1
