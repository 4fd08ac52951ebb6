#!/bin/bash
# An experiment build of libyavo.so with extra defines for one source (A/B on the same box via YAVO_LIB):
#   bash tools/build_variant.sh TAG SOURCE "-DNAME=VALUE ..."   -> ya_vo_amd/lib/libyavo_TAG.so
set -e
cd "$(dirname "$0")/../ya_vo_amd/csrc"
TAG=$1; SRC=$2; DEFS=$3
make -j16 >/dev/null
mkdir -p ../build/var_$TAG
EXTRA=""
[ "$SRC" = "yavo_kernels" ] && EXTRA="-mllvm -amdgpu-mfma-vgpr-form=1"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
    -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function $EXTRA $DEFS -c -o ../build/var_$TAG/$SRC.o $SRC.hip
OBJS=$(ls ../build/*.o | grep -v "/$SRC.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../lib/libyavo_$TAG.so $OBJS ../build/var_$TAG/$SRC.o -lz
echo "ya_vo_amd/lib/libyavo_$TAG.so"
