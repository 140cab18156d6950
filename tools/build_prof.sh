# dev build of libpcg with the int8 SCL phase profiler (-DPCG_SCLC_PROF) into altlib/
set -e
cd "$(dirname "$0")/.."
mkdir -p altlib
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-fast-math -Iinclude -Iantpolarcodes_amd/csrc"
/opt/rocm/bin/hipcc $F -DPCG_SCLC_PROF -c antpolarcodes_amd/csrc/scl_char_kernel.hip -o altlib/scl_char_prof.o
B=antpolarcodes_amd/csrc/build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $B/capi.cpp.o $B/plan.cpp.o $B/frames_capi.cpp.o $B/sc_kernel.hip.o $B/scl_kernel.hip.o $B/sclls_kernel.hip.o $B/frames_kernel.hip.o $B/sc_char_kernel.hip.o altlib/scl_char_prof.o -o altlib/libpcg_prof.so
