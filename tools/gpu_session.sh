set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06v; mkdir -p $O
TESTS="tests/test_gpu_c4_batch.py" ROUNDS=3 CONFIGS="c4 c4pull c5" EXTRA="--no-host-floor" timeout -k 10 1100 bash tools/ab.sh r06v_mm base g16384 g32768 > $O/ab.log 2>&1
