#!/bin/bash
# Build an A/B variant of liblio_gpu.so (CPU side): one source recompiled with extra defines, linked
# with the other objects of the current build, into fast-lio-sam_gps_amd/build_ab/<name>/liblio_gpu.so
# (select it on the GPU box with LIO_GPU_LIB=...).  usage: scripts/lib_ab.sh <name> <csrc file> <-Ddefines...>
set -eu
cd "$(dirname "$0")/../fast-lio-sam_gps_amd"
name=$1; src=$2; shift 2
d=build_ab/$name; mkdir -p "$d"
obj=$(basename "${src%.*}").o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -I../include -Icsrc \
    -D__HIP_PLATFORM_AMD__ "$@" -x hip -c "$src" -o "$d/$obj"
objs=$(ls build/*.o | grep -v "/$obj\$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$d/liblio_gpu.so" $objs "$d/$obj" -ldl -lpthread
echo "built $d/liblio_gpu.so"
