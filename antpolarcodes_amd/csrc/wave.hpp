// wave.hpp -- wave64 helpers shared by the CDNA4 decoder kernels.
#pragma once
#include <hip/hip_runtime.h>
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

PCG_DEV uint32_t fbits(float x) { return __float_as_uint(x); }
PCG_DEV float ubits(uint32_t u) { return __uint_as_float(u); }
PCG_DEV uint32_t sgn(float x) { return __float_as_uint(x) & 0x80000000u; }
PCG_DEV float fxor(float a, uint32_t s) { return __uint_as_float(__float_as_uint(a) ^ s); }
PCG_DEV float fabs_(float a) { return __uint_as_float(__float_as_uint(a) & 0x7fffffffu); }
// _mm256_min_ps / _mm256_max_ps semantics: the second operand on ties and NaN
PCG_DEV float minps(float a, float b) { return a < b ? a : b; }
PCG_DEV float maxps(float a, float b) { return a > b ? a : b; }

// f: sign(a)^sign(b) | min(|a|,|b|)          avx_float.h:55-63
PCG_DEV float polar_f(float a, float b)
{
    return ubits(((fbits(a) ^ fbits(b)) & 0x80000000u) | fbits(minps(fabs_(a), fabs_(b))));
}
// g: (a ^ signbit) + b                       avx_float.h:71-81
PCG_DEV float polar_g(float a, float b, uint32_t signbit) { return fxor(a, signbit) + b; }

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
