// wave.hpp -- wave64 helpers shared by the CDNA4 decoder kernels.
#pragma once
#ifndef PCG_RTC
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

namespace pcg {

#define PCG_DEV __device__ __forceinline__

PCG_DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Order this wave's LDS traffic: the DS unit executes one wave's instructions in
// order, so a compiler barrier + wave barrier is all that is needed between phases
// in which lanes exchange data through the wave's private LDS slice.
PCG_DEV void wsync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Read-only schedule words through the constant address space: uniform indices then
// become scalar loads (s_load, scalar cache) instead of vector loads on every op.
typedef const __attribute__((address_space(4))) uint32_t cu32_t;
PCG_DEV uint32_t ld_const(const uint32_t* p, uint32_t i)
{
    return reinterpret_cast<cu32_t*>(reinterpret_cast<uintptr_t>(p))[i];
}

PCG_DEV uint32_t fbits(float x) { return __float_as_uint(x); }
PCG_DEV float ubits(uint32_t u) { return __uint_as_float(u); }
PCG_DEV uint32_t sgn(float x) { return __float_as_uint(x) & 0x80000000u; }
PCG_DEV float fxor(float a, uint32_t s) { return __uint_as_float(__float_as_uint(a) ^ s); }
PCG_DEV float fabs_(float a) { return __uint_as_float(__float_as_uint(a) & 0x7fffffffu); }
// _mm256_min_ps / _mm256_max_ps semantics: the second operand on ties and NaN
PCG_DEV float minps(float a, float b) { return a < b ? a : b; }
PCG_DEV float maxps(float a, float b) { return a > b ? a : b; }

// f: sign(a)^sign(b) | min(|a|,|b|)          avx_float.h:55-63
// MINPS semantics (the second operand on ties and NaN): the compare takes abs source modifiers
// and the select picks the SIGNED operand whose magnitude wins, so the sign merge is one bit
// select -- v_cmp_lt |a|,|b|; v_cndmask; v_xor; v_bfi (4 VALU; selecting |a| / |b| instead
// made the compiler add a v_and per element: 5)
#ifndef PCG_F_OLD
#define PCG_F_OLD 0 // dev A/B: 1 = the round-4 formulation (abs values selected: 5 VALU)
#endif
PCG_DEV float polar_f(float a, float b)
{
#if PCG_F_OLD
    const float aa = __builtin_fabsf(a), ab = __builtin_fabsf(b);
    return ubits(((fbits(a) ^ fbits(b)) & 0x80000000u) | fbits(aa < ab ? aa : ab));
#endif
    const uint32_t ua = fbits(a), ub = fbits(b);
    const uint32_t sel = __builtin_fabsf(a) < __builtin_fabsf(b) ? ua : ub;
    // S2 ? S0 : S1 with S2 = the sign mask: the sign of a ^ b, the rest of sel (truth table
    // 0xE4: bit i = f(S0 = i>>2 & 1, S1 = i>>1 & 1, S2 = i & 1), the convention of 0x78 below)
    // (written as the builtin: the compiler turns the plain expression back into and + and_or)
    return ubits(__builtin_amdgcn_bitop3_b32(ua ^ ub, sel, 0x80000000u, 0xE4));
}
// g: (a ^ signbit) + b                       avx_float.h:71-81
PCG_DEV float polar_g(float a, float b, uint32_t signbit) { return fxor(a, signbit) + b; }
// g with the sign flip = bit k (< 32) of w: the bit shifted to the sign position and applied
// with one v_bitop3 (a ^ (t & 0x80000000); truth table 0x78 = S0 ^ (S1 & S2))
PCG_DEV float polar_g_bit(float a, float b, uint32_t w, uint32_t k)
{
    return ubits(__builtin_amdgcn_bitop3_b32(fbits(a), w << (31u - k), 0x80000000u, 0x78)) + b;
}

template <typename T>
PCG_DEV T shfl(T v, int src)
{
    return __shfl(v, src, 64);
}

PCG_DEV uint64_t ballot(bool p) { return __ballot(p); }

// XOR-reduce a 32-bit value across the wave
PCG_DEV uint32_t wave_xor(uint32_t v)
{
    for (int d = 32; d >= 1; d >>= 1)
        v ^= __shfl_xor(v, d, 64);
    return v;
}

// (value, index) argmin across the wave: smallest value, ties -> smallest index.
PCG_DEV void wave_argmin(float& v, uint32_t& i)
{
    for (int d = 32; d >= 1; d >>= 1) {
        float ov = __shfl_xor(v, d, 64);
        uint32_t oi = __shfl_xor(i, d, 64);
        if (ov < v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

// (value, index) argmax across the wave: largest value, ties -> smallest index.
PCG_DEV void wave_argmax(float& v, uint32_t& i)
{
    for (int d = 32; d >= 1; d >>= 1) {
        float ov = __shfl_xor(v, d, 64);
        uint32_t oi = __shfl_xor(i, d, 64);
        if (ov > v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

// Polar transform stages B = 1..16 (B < N) inside one 32-bit word of packed bits:
// x[i] ^= x[i + B] for positions with bit B clear (LSB-first packing).
PCG_DEV uint32_t transform_word(uint32_t w, uint32_t N)
{
    if (N > 1) w ^= (w >> 1) & 0x55555555u;
    if (N > 2) w ^= (w >> 2) & 0x33333333u;
    if (N > 4) w ^= (w >> 4) & 0x0F0F0F0Fu;
    if (N > 8) w ^= (w >> 8) & 0x00FF00FFu;
    if (N > 16) w ^= (w >> 16) & 0x0000FFFFu;
    return w;
}

// ---- packed codeword bits in LDS: position p -> word p>>5, bit p&31 ----------------
PCG_DEV uint32_t get_bit(const uint32_t* w, uint32_t p) { return (w[p >> 5] >> (p & 31)) & 1u; }

// Lanes 0..c-1 hold the bits of positions [o, o+c); c is 64, 32 or < 32 (then
// [o, o+c) lies inside one word).  Lane 0 stores.
PCG_DEV void put_bits(uint32_t* w, uint32_t o, uint32_t c, bool bit)
{
    const uint64_t m = ballot(bit);
    if (lane_id() == 0) {
        if (c >= 64) {
            w[o >> 5] = (uint32_t)m;
            w[(o >> 5) + 1] = (uint32_t)(m >> 32);
        } else if (c == 32) {
            w[o >> 5] = (uint32_t)m;
        } else {
            const uint32_t sh = o & 31, msk = ((1u << c) - 1u) << sh;
            const uint32_t old = w[o >> 5];
            w[o >> 5] = (old & ~msk) | (((uint32_t)m << sh) & msk);
        }
    }
}

} // namespace pcg

namespace pcg {

// ---- DPP / permlane butterflies (no LDS traffic) ------------------------------------
// Partner of lane i at distance d in a butterfly over aligned groups of 2d lanes.
// d = 1, 2: quad_perm xor; d = 4: row_half_mirror (i <-> 7-i); d = 8: row_mirror
// (i <-> 15-i); d = 16: v_permlane16_swap; d = 32: v_permlane32_swap.  The mirror
// partners are not xor partners, which is fine for commutative, idempotent combines
// (min / max / argmin / argmax / xor-after-uniformity is NOT idempotent: see xor below).
template <int D>
PCG_DEV uint32_t bfly(uint32_t v)
{
    if constexpr (D == 1)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false); // [1,0,3,2]
    else if constexpr (D == 2)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false); // [2,3,0,1]
    else if constexpr (D == 4)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x141, 0xF, 0xF, false); // row_half_mirror
    else if constexpr (D == 8)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x140, 0xF, 0xF, false); // row_mirror
    else if constexpr (D == 16) {
        auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
        return (lane_id() & 16) ? r[0] : r[1];
    } else {
        auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
        return (lane_id() & 32) ? r[0] : r[1];
    }
}

template <int D>
PCG_DEV float bflyf(float v)
{
    return ubits(bfly<D>(fbits(v)));
}

template <int D>
PCG_DEV void argmin_step(float& v, uint32_t& i)
{
    const float ov = bflyf<D>(v);
    const uint32_t oi = bfly<D>(i);
    if (ov < v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
    }
}

// argmin over aligned groups of g lanes (g power of two <= 64); every lane of the
// group ends with (min value, lowest index among equals).  Each level is a
// compile-time DPP/permlane op behind one uniform branch.
PCG_DEV void grp_argmin(float& v, uint32_t& i, uint32_t g)
{
    if (g > 1) argmin_step<1>(v, i);
    if (g > 2) argmin_step<2>(v, i);
    if (g > 4) argmin_step<4>(v, i);
    if (g > 8) argmin_step<8>(v, i);
    if (g > 16) argmin_step<16>(v, i);
    if (g > 32) argmin_step<32>(v, i);
}

template <int D>
PCG_DEV void argmax_step(float& v, uint32_t& i)
{
    const float ov = bflyf<D>(v);
    const uint32_t oi = bfly<D>(i);
    if (oi != 0xffffffffu && (i == 0xffffffffu || ov > v || (ov == v && oi < i))) {
        v = ov;
        i = oi;
    }
}

// argmax over the whole wave: (max value, lowest index among equals); `i == ~0` marks
// an empty lane that never wins.
PCG_DEV void wave_argmax_dpp(float& v, uint32_t& i)
{
    argmax_step<1>(v, i);
    argmax_step<2>(v, i);
    argmax_step<4>(v, i);
    argmax_step<8>(v, i);
    argmax_step<16>(v, i);
    argmax_step<32>(v, i);
}

// Exact xor partner: value of lane (i ^ J) for J in {1,2,4,8,16,32}.
template <int J>
PCG_DEV uint32_t xpartner(uint32_t v)
{
    if constexpr (J == 1)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0xB1, 0xF, 0xF, false);
    else if constexpr (J == 2)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x4E, 0xF, 0xF, false);
    else if constexpr (J == 4) {
        // lanes with bit 2 clear read lane i+4 (row_shl:4), the others lane i-4 (row_shr:4)
        const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x104, 0xF, 0xF, false);
        const uint32_t dn = (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x114, 0xF, 0xF, false);
        return (lane_id() & 4) ? dn : up;
    } else if constexpr (J == 8)
        return (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, 0x128, 0xF, 0xF, false); // row_ror:8
    else
        return bfly<J>(v); // permlane16/32 swaps are exact xor partners
}

// XOR over aligned groups of g lanes.  Mirror partners are fine: after the d-step
// every lane of a 2d-group holds the XOR of its d-group.
PCG_DEV uint32_t grp_xor(uint32_t v, uint32_t g)
{
    if (g > 1) v ^= bfly<1>(v);
    if (g > 2) v ^= bfly<2>(v);
    if (g > 4) v ^= bfly<4>(v);
    if (g > 8) v ^= bfly<8>(v);
    if (g > 16) v ^= bfly<16>(v);
    if (g > 32) v ^= bfly<32>(v);
    return v;
}

} // namespace pcg
