# dev builds of libpcg with the float SCL kernel at other occupancy targets (altlib/)
set -e
cd "$(dirname "$0")/.."
mkdir -p altlib
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-fast-math -Iinclude -Iantpolarcodes_amd/csrc"
B=antpolarcodes_amd/csrc/build
for m in ${MINWS:-3 4}; do
  /opt/rocm/bin/hipcc $F -DPCG_LS_MINW=$m -c antpolarcodes_amd/csrc/sclls_kernel.hip -o altlib/sclls_m$m.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $B/capi.cpp.o $B/plan.cpp.o $B/frames_capi.cpp.o $B/sc_kernel.hip.o $B/scl_kernel.hip.o altlib/sclls_m$m.o $B/frames_kernel.hip.o $B/sc_char_kernel.hip.o $B/scl_char_kernel.hip.o -o altlib/libpcg_m$m.so
done
