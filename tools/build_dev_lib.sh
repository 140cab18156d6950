#!/bin/bash
# Build a variant libpcg with extra compile flags for one kernel source into lib_dev/
# (development aid; select it with PCG_DEV_LIB=lib_dev/libpcg_<tag>.so).
#   [EXCL="<obj> ..."] [LP=8] [SKIP_MAKE=1] bash tools/build_dev_lib.sh <tag> <kernel.hip> <flags...>
# (SKIP_MAKE: the in-tree objects are current; lets several variants build in parallel)
# sclls_kernel.hip: the variant is one list width (LP, default 8) plus the host part, replacing
# the objects sclls_kernel.hip.o and sclls_lp<LP>.o; its specialised (hiprtc) kernels carry the
# same -D knobs (sclls_rtc_defines).  Plans of the other list widths are refused by such a library
# (PCG_E_UNSUPPORTED at creation: their objects were built with the default knobs).
set -e
TAG=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/antpolarcodes_amd/csrc
[ -n "$SKIP_MAKE" ] || make -s -C "$CS" -j8 >/dev/null
mkdir -p "$ROOT/lib_dev"
EXTRA=()
if [ "$SRC" = sclls_kernel.hip ]; then
  EXTRA=(-DPCG_LS_INST=${LP:-8} -DPCG_LS_HOST)
  EXCL=${EXCL:-"sclls_kernel.hip sclls_lp${LP:-8}"}
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
    -fno-fast-math -I"$ROOT/include" -I"$CS" "${EXTRA[@]}" "$@" -c "$CS/$SRC" -o "/tmp/dev_$TAG.o"
OBJS=$(ls "$CS"/build/*.o)
for x in ${EXCL:-$SRC}; do OBJS=$(echo "$OBJS" | grep -v "/$x.o$"); done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $OBJS "/tmp/dev_$TAG.o" -o "$ROOT/lib_dev/libpcg_$TAG.so" -ldl
echo "lib_dev/libpcg_$TAG.so"
