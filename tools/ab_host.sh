# same-box A/B of a host-side change on C1: the current build against
# tools/variants/$2 (built from the previous commit), alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${1:-abh}; mkdir -p $O
for r in 1 2 3; do
  for v in cur $2; do
    if [ $v = cur ]; then unset PSF_LIBRARY_VARIANT; else export PSF_LIBRARY_VARIANT=tools/variants/$v/libpsf.so; fi
    timeout -k 10 200 python bench.py --config c1 --no-cpu-baseline --steps 200 > $O/c1_${v}_$r.json 2> $O/c1_${v}_$r.err || { tail -20 $O/c1_${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['host']; print(sys.argv[2], d['value'], d['ms_per_step'], 'active', h['active_ms_per_step'], 'kernel', h['kernel_ms_per_step'])" $O/c1_${v}_$r.json "$v"
  done
done
