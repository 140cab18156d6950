#!/bin/bash
# Build a variant libpcg with extra compile flags for one kernel source into lib_dev/
# (development aid; select it with PCG_DEV_LIB=lib_dev/libpcg_<tag>.so).
#   [EXCL=<replaced.hip>] [SKIP_MAKE=1] bash tools/build_dev_lib.sh <tag> <kernel.hip> <flags...>
# (SKIP_MAKE: the in-tree objects are current; lets several variants build in parallel)
set -e
TAG=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/antpolarcodes_amd/csrc
[ -n "$SKIP_MAKE" ] || make -s -C "$CS" -j8 >/dev/null
mkdir -p "$ROOT/lib_dev"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
    -fno-fast-math -I"$ROOT/include" -I"$CS" "$@" -c "$CS/$SRC" -o "/tmp/dev_$TAG.o"
OBJS=$(ls "$CS"/build/*.o | grep -v "/${EXCL:-$SRC}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $OBJS "/tmp/dev_$TAG.o" -o "$ROOT/lib_dev/libpcg_$TAG.so"
echo "lib_dev/libpcg_$TAG.so"
