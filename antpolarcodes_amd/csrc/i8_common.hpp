// i8_common.hpp -- int8 ("char") building blocks shared by the lane-serial 8-bit kernels
// (scl_char_kernel.hip: SclFipChar, sccs_kernel.hip: FastSscFipChar): the reference's byte
// arithmetic (fip_char.h) on packed dwords, 16-byte lane-column stage units and their sources.
#pragma once
#include "wave.hpp"

namespace pcg {
namespace i8 {

PCG_DEV int sat8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }
PCG_DEV int sbyte(uint32_t d, uint32_t b) { return (int)(int8_t)(uint8_t)(d >> (8 * b)); }
PCG_DEV uint32_t ubyte(int v, uint32_t b) { return ((uint32_t)v & 0xffu) << (8 * b); }

// FastSscFip::F_function_calc / G_function_calc (fip_char.h:35-64)
PCG_DEV int fip_f(int l, int r)
{
    const bool neg = (l ^ r) < 0;
    int a = l > -127 ? l : -127, b = r > -127 ? r : -127;
    a = a < 0 ? -a : a;
    b = b < 0 ? -b : b;
    a = a > 1 ? a : 1;
    b = b > 1 ? b : 1;
    const int m = a < b ? a : b;
    return neg ? -m : m;
}
PCG_DEV int fip_g(int l, int r, uint32_t bit) { return sat8(bit ? r - l : r + l); }

// ---- 4 bytes per dword with packed 16-bit ops ----------------------------------------
// Each byte is placed in the high byte of a 16-bit lane (low byte 0): even bytes (0, 2)
// and odd bytes (1, 3) form two v_pk_*_i16 pairs.  In this form int16 saturation is the
// reference's int8 saturation (_mm256_adds_epi8 / subs_epi8) and the result byte is the
// high byte of each lane.
typedef short s2_t __attribute__((ext_vector_type(2)));
PCG_DEV s2_t as_s2(uint32_t x) { return __builtin_bit_cast(s2_t, x); }
PCG_DEV uint32_t as_u(s2_t x) { return __builtin_bit_cast(uint32_t, x); }
PCG_DEV uint32_t hb_even(uint32_t a) { return __builtin_amdgcn_perm(0u, a, 0x020c000cu); }
PCG_DEV uint32_t hb_odd(uint32_t a) { return a & 0xff00ff00u; }
PCG_DEV uint32_t hb_pack(uint32_t even, uint32_t odd) { return __builtin_amdgcn_perm(odd, even, 0x07030501u); }

// F_function_calc (fip_char.h:35-56): sign(l)^sign(r) * max(1, min(|max(l,-127)|, |max(r,-127)|))
PCG_DEV uint32_t f_pair(uint32_t l, uint32_t r)
{
    const s2_t a = as_s2(l), b = as_s2(r), z = { 0, 0 };
    const s2_t aa = __builtin_elementwise_max(a, __builtin_elementwise_sub_sat(z, a));
    const s2_t ab = __builtin_elementwise_max(b, __builtin_elementwise_sub_sat(z, b));
    s2_t m = __builtin_elementwise_min(aa, ab);
    m = __builtin_elementwise_min(m, (s2_t){ 0x7f00, 0x7f00 }); // |max(x, -127)| = min(|x|, 127)
    m = __builtin_elementwise_max(m, (s2_t){ 0x100, 0x100 });
    const s2_t sg = as_s2(l ^ r) >> (s2_t){ 15, 15 };
    return as_u(as_s2(as_u(m) ^ as_u(sg)) - sg);
}
PCG_DEV uint32_t f4(uint32_t a, uint32_t b)
{
    return hb_pack(f_pair(hb_even(a), hb_even(b)), f_pair(hb_odd(a), hb_odd(b)));
}
// G_function_calc (fip_char.h:58-64): bit ? sat(r - l) : sat(r + l); `bits` bit k <-> byte k
PCG_DEV uint32_t g_pair(uint32_t l, uint32_t r, uint32_t msk)
{
    const s2_t a = as_s2(l), b = as_s2(r);
    const uint32_t sum = as_u(__builtin_elementwise_add_sat(b, a)), dif = as_u(__builtin_elementwise_sub_sat(b, a));
    return (dif & msk) | (sum & ~msk);
}
PCG_DEV uint32_t bitmask2(uint32_t bits, uint32_t k0)
{ // 16-bit lane masks from bits k0 and k0 + 2
    const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)bits, k0, 1);
    const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)bits, k0 + 2, 1);
    return (m0 & 0x0000ffffu) | (m1 & 0xffff0000u);
}
PCG_DEV uint32_t g4b(uint32_t a, uint32_t b, uint32_t bits, uint32_t k0)
{
    return hb_pack(g_pair(hb_even(a), hb_even(b), bitmask2(bits, k0)),
                   g_pair(hb_odd(a), hb_odd(b), bitmask2(bits, k0 + 1)));
}
PCG_DEV uint32_t g4(uint32_t a, uint32_t b, uint32_t nib) { return g4b(a, b, nib, 0); }
// sums over the 4 signed bytes of a dword: sum of x and sum of |x| (v_dot4 / v_sad_u8)
PCG_DEV int bsum(uint32_t a) { return __builtin_amdgcn_sdot4((int)a, 0x01010101, 0, false); }
PCG_DEV int babs(uint32_t a) { return (int)__builtin_amdgcn_sad_u8(a ^ 0x80808080u, 0x80808080u, 0u); }
// sign bits of 4 bytes as a nibble
PCG_DEV uint32_t sign4(uint32_t d)
{
    return ((d >> 7) & 1u) | ((d >> 14) & 2u) | ((d >> 21) & 4u) | ((d >> 28) & 8u);
}

// 16 x int8 per lane and unit
PCG_DEV uint4 f16(const uint4& a, const uint4& b)
{
#if defined(PCG_I8_ABL) && (PCG_I8_ABL & 1) // dev ablation (wrong results): F's byte arithmetic removed
    return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
#endif
    return make_uint4(f4(a.x, b.x), f4(a.y, b.y), f4(a.z, b.z), f4(a.w, b.w));
}
PCG_DEV uint4 g16(const uint4& a, const uint4& b, uint32_t bits16)
{
#if defined(PCG_I8_ABL) && (PCG_I8_ABL & 2) // dev ablation (wrong results): G's byte arithmetic removed
    return make_uint4(a.x ^ b.x ^ bits16, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
#endif
    return make_uint4(g4b(a.x, b.x, bits16, 0), g4b(a.y, b.y, bits16, 4), g4b(a.z, b.z, bits16, 8),
                      g4b(a.w, b.w, bits16, 12));
}
PCG_DEV uint32_t dw_of(const uint4& v, uint32_t k) { return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w)); }
PCG_DEV int byte_of(const uint4& v, uint32_t i) { return sbyte(dw_of(v, i >> 2), i & 3u); }
// sign bits of 16 bytes
PCG_DEV uint32_t sign16(const uint4& v)
{
    return sign4(v.x) | (sign4(v.y) << 4) | (sign4(v.z) << 8) | (sign4(v.w) << 12);
}

// Stage s >= 4 occupies 2^s / 16 units of 16 bytes per lane, unit c of lane l at
// [(base(s) + c) * 64 + l] (uint4), so a wave-wide unit access is one contiguous 1 KiB;
// stages 0..3 share unit 0 (stage t at bytes [2^t, 2^(t+1))) and always live in LDS.
__host__ __device__ inline uint32_t st_units(uint32_t s) { return s <= 3 ? (s ? 1u : 0u) : (1u << (s - 4)); }
__host__ __device__ inline uint32_t st_base(uint32_t s) { return s <= 3 ? 0u : (1u << (s - 4)); }


// _mm256_adds_epi8 on 16 bytes
PCG_DEV uint32_t adds4(uint32_t a, uint32_t b)
{
    const uint32_t e = as_u(__builtin_elementwise_add_sat(as_s2(hb_even(a)), as_s2(hb_even(b))));
    const uint32_t o = as_u(__builtin_elementwise_add_sat(as_s2(hb_odd(a)), as_s2(hb_odd(b))));
    return hb_pack(e, o);
}
PCG_DEV uint4 adds16(const uint4& a, const uint4& b)
{
    return make_uint4(adds4(a.x, b.x), adds4(a.y, b.y), adds4(a.z, b.z), adds4(a.w, b.w));
}

// quantise 4 floats as CharContainer::insertLlr does (bitcontainer.cpp:449-516)
PCG_DEV uint32_t quant4(const float4& v, bool large)
{
    const float x[4] = { v.x, v.y, v.z, v.w };
    uint32_t o = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
        int q;
        if (large) { // convert_f32_to_int8_large: cvtps_epi32 (NaN, |x| >= 2^31 -> INT_MIN) + packs
            if (!(x[k] < 2147483648.0f) || x[k] < -2147483648.0f) {
                q = -128;
            } else {
                const float r = __builtin_rintf(x[k]);
                q = r <= -128.0f ? -128 : (r >= 127.0f ? 127 : (int)r);
            }
        } else { // vectorizedFtoC (8 <= N < 32)
            float t = x[k] > -128.0f ? x[k] : -128.0f;
            t = t < 127.0f ? t : 127.0f;
            q = (int)__builtin_rintf(t);
        }
        o |= ubyte(q, k);
    }
    return o;
}

// ---- stage sources: ld(c) = unit c (16 bytes) of the stage --------------------------
template <bool I8>
struct ChanSrc { // the channel frame (stage top)
    const void* y;
    uint32_t N;
    PCG_DEV uint4 ld(uint32_t c) const
    {
        if constexpr (I8) {
            if (N >= 16)
                return reinterpret_cast<const uint4*>(y)[c];
            const uint2 v = reinterpret_cast<const uint2*>(y)[0]; // N = 8
            return make_uint4(v.x, v.y, 0u, 0u);
        } else {
            const float4* f = reinterpret_cast<const float4*>(y) + 4u * c;
            const bool large = N >= 32;
            if (N >= 16)
                return make_uint4(quant4(f[0], large), quant4(f[1], large), quant4(f[2], large),
                                  quant4(f[3], large));
            return make_uint4(quant4(f[0], large), quant4(f[1], large), 0u, 0u);
        }
    }
};
// bytes [k, k+16) of a 32-byte window (lo, hi), k a multiple of 4 (N = 16 root split)
PCG_DEV uint4 shift_units(const uint4& lo, uint32_t k)
{
    const uint32_t d[4] = { lo.x, lo.y, lo.z, lo.w };
    const uint32_t q = k >> 2;
    return make_uint4(q + 0 < 4 ? d[(q + 0) & 3] : 0u, q + 1 < 4 ? d[(q + 1) & 3] : 0u,
                      q + 2 < 4 ? d[(q + 2) & 3] : 0u, q + 3 < 4 ? d[(q + 3) & 3] : 0u);
}
template <bool I8>
struct RootSrc { // stage top-1, recomputed: F (left child) or G with the own left-half bits
    ChanSrc<I8> ch;
    const uint32_t* row; // own bit row, word w at [w * 64]
    uint32_t mode;       // 0: F (left child), 1: G (right child), 2: saturating sum (ZeroRNode's G_0R)
    PCG_DEV uint4 ld(uint32_t c) const
    {
        const uint32_t N = ch.N;
        uint4 a, b;
        if (N >= 32) {
            a = ch.ld(c);
            b = ch.ld(c + (N >> 5));
        } else { // N = 8 / 16: the whole frame is in unit 0
            a = ch.ld(0);
            b = shift_units(a, N >> 1);
        }
        if (mode == 0)
            return f16(a, b);
        if (mode == 2)
            return adds16(a, b);
        const uint32_t p0 = 16u * c;
        const uint32_t w = row[(p0 >> 5) << 6];
        return g16(a, b, (w >> (p0 & 31u)) & 0xffffu);
    }
};
// 128-bit byte shifts (k = 1, 2, 4, 8)
PCG_DEV uint4 shr_bytes(const uint4& v, uint32_t k)
{
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    const uint32_t b = 8u * k;
    const uint64_t rl = k >= 8 ? hi : ((lo >> b) | (hi << (64u - b))), rh = k >= 8 ? 0ull : (hi >> b);
    return make_uint4((uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32));
}
PCG_DEV uint4 shl_bytes(const uint4& v, uint32_t k)
{
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    const uint32_t b = 8u * k;
    const uint64_t rh = k >= 8 ? lo : ((hi << b) | (lo >> (64u - b))), rl = k >= 8 ? 0ull : (lo << b);
    return make_uint4((uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32));
}
struct SmallSrc { // stages 0..3: bytes [2^s, 2^(s+1)) of the shared unit
    const uint4* b;
    uint32_t l, k; // k = 2^s
    PCG_DEV uint4 ld(uint32_t) const { return shr_bytes(b[l], k); }
};
struct SmallDst {
    uint4* b;
    uint32_t l, k;
    PCG_DEV void st(uint32_t, const uint4& v) const
    {
        const uint4 u = b[l], x = shl_bytes(v, k);
        // byte mask of [k, 2k)
        const uint64_t ml = k >= 8 ? 0ull : (((k >= 4 ? 0xffffffffull : ((1ull << (8u * k)) - 1ull))) << (8u * k));
        const uint64_t mh = k >= 8 ? ~0ull : 0ull;
        const uint64_t ul = ((uint64_t)u.y << 32) | u.x, uh = ((uint64_t)u.w << 32) | u.z;
        const uint64_t xl = ((uint64_t)x.y << 32) | x.x, xh = ((uint64_t)x.w << 32) | x.z;
        const uint64_t rl = (ul & ~ml) | (xl & ml), rh = (uh & ~mh) | (xh & mh);
        b[l] = make_uint4((uint32_t)rl, (uint32_t)(rl >> 32), (uint32_t)rh, (uint32_t)(rh >> 32));
    }
};
struct LdsSrc {
    const uint4* b; // stage base
    uint32_t l;     // lane column
    PCG_DEV uint4 ld(uint32_t c) const { return b[(c << 6) + l]; }
};
struct GlbSrc {
    const uint4* b;
    uint32_t l;
    PCG_DEV uint4 ld(uint32_t c) const { return b[((uint64_t)c << 6) + l]; }
};
struct LdsDst {
    uint4* b;
    uint32_t l;
    PCG_DEV void st(uint32_t c, const uint4& v) const { b[(c << 6) + l] = v; }
};
struct GlbDst {
    uint4* b;
    uint32_t l;
    PCG_DEV void st(uint32_t c, const uint4& v) const { b[((uint64_t)c << 6) + l] = v; }
};

} // namespace i8
} // namespace pcg
