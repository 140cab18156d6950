// kernels.hpp -- device launch interface shared by the C ABI and the kernels.
#pragma once
#ifndef PCG_RTC
#include <hip/hip_runtime.h>
#include <stdlib.h>
#endif
#include <stdint.h>

namespace pcg {

struct KernelArgs {
    const float* llr;         // F x N channel LLRs (device)
    uint64_t F;
    const uint32_t* ops;      // flattened schedule (device)
    uint32_t nops;
    uint32_t N, log2N, K, kb, L;
    const uint16_t* info_pos; // K info positions (device)
    const uint32_t* crc_m;    // K syndrome columns (device)
    uint32_t crc_c0;
    uint32_t crc_bits;        // 0, 8, 11, 16, 32
    const uint32_t* crc_rows; // crc_bits x W codeword masks (device): syndrome bit r = c0_r ^ parity(cw & row r)
    int systematic;
    uint8_t* info;            // F x kb (device)
    uint8_t* ok;              // F or null
    float* metrics;           // F x L or null (SCL)
    uint32_t wave_lds_floats; // LDS floats per wave (codeword)
    float* scratch;           // global per-codeword scratch (SCL large stages)
    uint64_t scratch_floats;  // per codeword
    uint32_t lds_stage_limit; // SCL: stages < limit live in LDS
    unsigned long long* prof; // dev-only: per-op-code [cycles, count] (null = off)
    uint32_t flags;           // dev-only experiment switches (PCG_FLAGS), 0 in production
    uint32_t scl_virt;        // lane-serial SCL: top stages recomputed instead of stored (0..2)
    uint32_t scl_fuse;        // lane-serial SCL: bit 0 F/G + child F fused over global stages, bit 1 idle lanes share F/G, bit 2 root-child ops stage the channel in LDS (PCG_SCL_FUSE)
    // lane-serial SCL only: decode frames fmap[0 .. *fcount) (device) instead of 0 .. F-1
    // (the adaptive decoder's second stage; F bounds *fcount and sizes the grid)
    const uint32_t* fmap;
    const uint32_t* fcount;
    // 8-bit ("char") plans: F x N int8 channel LLRs; null -> `llr` floats are quantised
    // in the kernel exactly as CharContainer::insertLlr does
    const int8_t* llr8;
    // persistent lane-serial kernels: a device counter the caller zeroes on the launch
    // stream before every launch (capi.cpp); waves take codeword groups from it (dynamic
    // balance across SIMDs whose wave counts differ).  null -> static grid-stride assignment.
    uint32_t* queue;
    // grid size (persistent waves) chosen by the caller: min(groups, the plan's wave cap)
    uint32_t units;
    // SCL: initial path-0 metric of every frame (0 = a freshly constructed decoder; the
    // previous frame's final path-0 metric reproduces the reference's carry across frames of
    // one decoder instance)
    float metric0;
    // Fast-SSC (sc_kernel.hip): F x N soft codeword output (Decoder::getSoftCodeword) or null
    float* soft;
    // lane-serial SCL: lanes per codeword (a power of two >= the list size rounded up; 0 =
    // that minimum).  Wider groups give the idle lanes F/G work (ls_share): the adaptive
    // decoder's second stage, a few frames at a time, runs latency-bound walks.
    uint32_t scl_lp;
    // lane-serial SCL: stages 3 .. 2+scl_v3 are recomputed wherever they are read (sclls_layout)
    uint32_t scl_v3;
    // lane-serial SCL with lazy bit buffers (LP >= PCG_LS_DBITS_LP): D[4 .. scl_sb-1] in LDS,
    // the rest in the global slab; 0 for the per-lane codeword rows of smaller LP
    uint32_t scl_sb;
    // lane-serial SCL on punctured frames (pcg_decode_punctured_f32): frame f's E = in_stride
    // received LLRs start at llr + f * in_stride, and position j of its depunctured codeword is
    // llr[pmap[j]], or +0.0 where pmap[j] < 0 (Puncturer::depuncture, puncturer.h:92-99).  Each
    // wave depunctures its codeword group into its scratch slab (scratch_floats includes the
    // G x N region).  null: the frames are N LLRs each.
    const int32_t* pmap;
    uint32_t in_stride;
};

#ifndef PCG_RTC
// PCG_*_WPC developer overrides of the waves per CU: ignored unless a positive number
inline uint64_t env_wpc(const char* name, uint64_t dflt)
{
    if (const char* e = getenv(name)) {
        const long v = strtol(e, nullptr, 10);
        if (v > 0 && v <= 64)
            return (uint64_t)v;
    }
    return dflt;
}
#endif

// Dynamic group assignment for the persistent lane-serial kernels (KernelArgs::queue;
// one-wave workgroups). Every lane gets the same ticket; a wave stops at its first ticket
// past the last group.  The counter is reset by a hipMemsetAsync on the launch stream
// before each launch, so an aborted launch or another stream cannot leave it dirty.
__device__ inline uint64_t queue_next(uint32_t* q)
{
    uint32_t t = 0;
    if (__lane_id() == 0)
        t = __hip_atomic_fetch_add(q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
}

#ifndef PCG_RTC
// LDS floats one SC codeword needs: alpha (N floats, index 0 unused) + packed bits.
inline uint32_t sc_wave_lds_floats(uint32_t N) { return N + (N >= 64 ? N / 32 : 2) + 2; }

int launch_sc(const KernelArgs& a, hipStream_t stream); // one codeword per wave; a.soft: + soft codeword
uint32_t sc_soft_lds_bytes(uint32_t N);                  // 0: N too large for the soft-output decode
int launch_sc_char(const KernelArgs& a, hipStream_t stream);   // FastSscFipChar (sc_char_kernel.hip)
int launch_scl_char(const KernelArgs& a, hipStream_t stream);  // SclFipChar (scl_char_kernel.hip)
#endif // PCG_RTC

} // namespace pcg

#ifndef PCG_RTC
namespace pcg {
// Persistent lane-serial kernels: per-wave LDS / global scratch layout, the wave cap of a
// launch on the current device (CUs x resident waves per CU from hipOccupancy; evaluated
// once per plan), and the launch (grid = KernelArgs::units)
inline uint64_t wave_units(uint64_t F, uint32_t frames_per_wave, uint64_t cap)
{
    const uint64_t need = (F + frames_per_wave - 1) / frames_per_wave;
    return need < cap ? need : cap;
}
// lane-serial SCL kernel (sclls_kernel.hip), 64 / L' codewords per wave
int sclls_layout(uint32_t N, uint32_t L, uint32_t lp, uint32_t vleaf, uint32_t* wave_lds_floats,
                 uint32_t* lds_stage_limit, uint64_t* scratch_floats, uint32_t* virt, uint32_t* v3, uint32_t* sb);
uint64_t sclls_wave_cap(uint32_t lp, uint32_t wave_lds_floats);
int launch_sclls(const KernelArgs& a, hipStream_t stream);
// 8-bit SCL (scl_char_kernel.hip): LDS dwords per wave, LDS stage limit, global scratch dwords
int sclc_layout(uint32_t N, uint32_t L, uint32_t* lds_dwords, uint32_t* Sl, uint64_t* scratch_dwords);
uint64_t sclc_wave_cap(uint32_t L, uint32_t lds_dwords, bool i8);
// lane-serial Fast-SSC (scs_kernel.hip), 64 codewords per wave
int scs_layout(uint32_t N, uint32_t* lds_dwords, uint32_t* Sl, uint64_t* scratch_dwords);
uint64_t scs_wave_cap(uint32_t lds_dwords);
int launch_scs(const KernelArgs& a, hipStream_t stream);
// LDS-resident Fast-SSC (scq_kernel.hip), Q lanes per codeword: LDS dwords per wave (0: does
// not fit), wave cap, launch
uint32_t scq_layout(uint32_t N, uint32_t Q, bool V);
uint64_t scq_wave_cap(uint32_t Q, bool V, uint32_t lds_dwords);
int launch_scq(const KernelArgs& a, uint32_t Q, bool V, hipStream_t stream);
// lane-serial 8-bit Fast-SSC (sccs_kernel.hip), 64 codewords per wave
int sccs_layout(uint32_t N, uint32_t* lds_dwords, uint32_t* Sl, uint64_t* scratch_dwords);
uint64_t sccs_wave_cap(uint32_t lds_dwords, bool i8);
int launch_sccs(const KernelArgs& a, hipStream_t stream);
} // namespace pcg
#endif // PCG_RTC
