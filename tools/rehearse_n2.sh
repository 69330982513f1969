# N=2 rehearsal of the driver's scaling launch on one GPU (two ranks sharing
# cuda:0, gloo for the process group: PSF_SAME_GPU / PSF_DIST_BACKEND are the
# bench's rehearsal knobs), plus the C1 host-section profile (diagnostic
# build tools/variants/hprof).  Output: gpurun_out/$1/.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-rehearse}; mkdir -p $O
if [ -f tools/variants/hprof/libpsf.so ]; then
  timeout -k 10 150 python tools/host_prof.py > $O/hprof_c1.txt 2>&1 || exit 1
fi
p=29511
for c in c2 c4 c5; do
  extra=""; [ $c = c5 ] && extra="--compress"
  PSF_SAME_GPU=1 PSF_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $p bench.py --gpus 2 --config $c $extra --steps 5 --warmup 2 --no-cpu-baseline \
    > $O/n2_$c.json 2> $O/n2_$c.err || exit 1
  p=$((p + 1))
done
cat $O/hprof_c1.txt 2>/dev/null
for c in c2 c4 c5; do grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*\|"backend": "[a-z]*"' $O/n2_$c.json | tr '\n' ' '; echo; done
