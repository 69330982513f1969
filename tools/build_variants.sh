#!/bin/bash
# Tuning experiments: build libpsf.so variants of ff_codec.hip with -D knobs
# into tools/variants/<name>/ (git-ignored); load one with
# PSF_LIBRARY_VARIANT=tools/variants/<name>/libpsf.so.
#   tools/build_variants.sh <name> [flags...]      (SRC=<file> overrides the source)
set -e
cd "$(dirname "$0")/.."
python -m parameter_server_amd.build > /dev/null
SRCF=${SRC:-parameter_server_amd/csrc/ff_codec.hip}
EXCL=${EXCL:-$(basename $SRCF).o}
OBJS=$(ls parameter_server_amd/build/*.o | grep -v "/$EXCL$")
name=$1; shift
mkdir -p tools/variants/$name
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude -Iparameter_server_amd/csrc "$@" \
  -c $SRCF -o tools/variants/$name/variant.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/$name/libpsf.so $OBJS tools/variants/$name/variant.o
echo tools/variants/$name/libpsf.so
