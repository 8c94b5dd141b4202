#!/bin/bash
# Build an experimental variant of libconcrete_hip.so: tools/variant.sh NAME "-DFOO=1 ..."
# -> variants/libconcrete_hip_NAME.so (use with CONCRETE_HIP_LIB=...)
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/variants/build_$NAME
mkdir -p $B
cd $R/concrete_amd/csrc
make -s -j8 LIB=$R/variants/libconcrete_hip_$NAME.so OBJDIR=$B HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result $*" $R/variants/libconcrete_hip_$NAME.so
