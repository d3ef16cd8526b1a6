#!/bin/bash
# build a variant of the library with extra -D flags on lane_decode.hip:
#   tools/build_variant.sh NAME -DFOO=1 ...  ->  zlib-streams_amd/libzstreams_mi355x_NAME.so
# (SRC=chunk_kernels to vary that file instead)
set -e
N=$1; shift
cd "$(dirname "$0")/../zlib-streams_amd/csrc"
make -s
mkdir -p build_var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c ${SRC:-lane_decode}.hip -o build_var/${SRC:-lane_decode}_$N.o
OBJS=$(ls build/*.o | grep -v ${SRC:-lane_decode}.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,-Bsymbolic -o ../libzstreams_mi355x_$N.so $OBJS build_var/${SRC:-lane_decode}_$N.o
echo built ../libzstreams_mi355x_$N.so
