set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t2; mkdir -p $O


ROUNDS=4 CONFIGS="c1" EXTRA="--no-host-floor" timeout -k 10 900 bash tools/ab.sh r06t2_c1 base head > $O/ab.log 2>&1
