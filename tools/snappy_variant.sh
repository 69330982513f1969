#!/bin/bash
# A/B builds of the snappy kernels: tools/snappy_variant.sh <name> <snappy.hip>
# builds tools/variants/<name>/libpsf.so (git-ignored) from the current objects
# with <snappy.hip> in place of csrc/snappy.hip; load it with
# PSF_LIBRARY_VARIANT=tools/variants/<name>/libpsf.so.
set -e
cd "$(dirname "$0")/.."
python -m parameter_server_amd.build > /dev/null
name=$1; src=$2
mkdir -p tools/variants/$name
OBJS=$(ls parameter_server_amd/build/*.o | grep -v "/snappy.hip.o$")
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Iinclude \
  -Iparameter_server_amd/csrc -c "$src" -o tools/variants/$name/snappy.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/$name/libpsf.so $OBJS tools/variants/$name/snappy.o
echo tools/variants/$name/libpsf.so
