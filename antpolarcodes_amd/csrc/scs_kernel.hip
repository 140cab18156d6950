// scs_kernel.hip -- lane-serial batched Fast-SSC ("SC") polar decoding on CDNA4 (gfx950).
//
// Lane = one codeword: a wave decodes 64 frames at once, walking the plan's Fast-SSC
// schedule (plan.cpp sc_emit, the reference's FastSscAvx tree in decode order) uniformly
// while every lane runs the reference's scalar per-node loops on its own LLRs -- the
// same arithmetic, in the same order, as the AVX2 code (fastssc_avx_float.cpp; see
// oracle/polar_oracle.c, which this follows leaf for leaf).  Compared with the
// one-codeword-per-wave sc_kernel.hip this removes the cross-lane reductions, the
// per-node barriers and the idle lanes of small nodes.
//
// Per lane:
//   * LLR stages 1 <= s < top-1 as float4 units in a lane column (unit c of lane l at
//     [(base(s) + c) * 64 + l]: a wave-wide unit access is one contiguous 1 KiB), LDS for
//     s < Sl, a per-wave global slab above;
//   * stage top-1 (the root's children) recomputed from the channel frame wherever it is
//     read: F(y_i, y_i+N/2) while the left child is decoded, G(y_i, y_i+N/2, bit_i) with
//     the lane's own left-half bits afterwards;
//   * the codeword estimate as packed sign bits, one LDS word column per lane (only sign
//     bits of the reference's float "bits" are observable, as in sc_kernel.hip).
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"

#include <stdio.h>
#include <stdlib.h>

namespace pcg {

namespace {

constexpr float FLT_MAX_S = 3.40282347e+38f;

// ---- layout ---------------------------------------------------------------------------
// stage 1 (2 floats) takes one unit, stage s >= 2 takes 2^(s-2) units
__host__ __device__ inline uint32_t ss_base(uint32_t s) { return s >= 2 ? (1u << (s - 2)) : 0u; }

struct SsLayout {
    uint32_t Sl;      // stages < Sl in LDS
    uint32_t mt;      // recomputed stage (top-1)
    uint32_t bits;    // LDS dword offset of the bit rows (word w of lane l at [w * 64 + l])
    uint32_t lds;     // LDS dwords per wave
    uint64_t gdwords; // global slab dwords per wave
};

__host__ __device__ inline SsLayout ss_layout(uint32_t N, uint32_t Sl)
{
    SsLayout y;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    y.mt = top - 1;
    y.Sl = Sl < 1 ? 1 : (Sl > y.mt ? y.mt : Sl);
    y.bits = 256u * ss_base(y.Sl);
    const uint32_t W = N >= 32 ? N / 32 : 1u;
    y.lds = y.bits + 64u * W;
    y.gdwords = 256ull * (ss_base(y.mt) - ss_base(y.Sl));
    return y;
}

PCG_DEV float4 f4_f(const float4& a, const float4& b)
{
    return make_float4(polar_f(a.x, b.x), polar_f(a.y, b.y), polar_f(a.z, b.z), polar_f(a.w, b.w));
}
PCG_DEV float4 f4_g(const float4& a, const float4& b, uint32_t nib)
{
    return make_float4(polar_g(a.x, b.x, (nib & 1u) << 31), polar_g(a.y, b.y, ((nib >> 1) & 1u) << 31),
                       polar_g(a.z, b.z, ((nib >> 2) & 1u) << 31), polar_g(a.w, b.w, ((nib >> 3) & 1u) << 31));
}
PCG_DEV float4 f4_add(const float4& a, const float4& b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
PCG_DEV float f4_at(const float4& v, uint32_t k) { return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w)); }
PCG_DEV uint32_t sgn4(const float4& v)
{
    return (fbits(v.x) >> 31) | ((fbits(v.y) >> 31) << 1) | ((fbits(v.z) >> 31) << 2) | ((fbits(v.w) >> 31) << 3);
}

// ---- stage sources -------------------------------------------------------------------
struct ChanSrc {
    const float4* y;
    PCG_DEV float4 ld(uint32_t c) const { return y[c]; }
};
struct RootSrc { // stage top-1, recomputed
    const float4* y;
    uint32_t half;       // N/8 units
    const uint32_t* row; // own bit row, word w at [w * 64]
    uint32_t mode;       // 0: F (left child), 1: G (right child), 2: G0 (right child of ZeroRNode)
    PCG_DEV float4 ld(uint32_t c) const
    {
        const float4 a = y[c], b = y[c + half];
        if (mode == 0)
            return f4_f(a, b);
        if (mode == 2)
            return f4_add(a, b);
        const uint32_t p0 = 4u * c;
        return f4_g(a, b, (row[(p0 >> 5) << 6] >> (p0 & 31u)) & 0xfu);
    }
};
struct LdsSrc {
    const float4* b;
    PCG_DEV float4 ld(uint32_t c) const { return b[c << 6]; }
};
struct GlbSrc {
    const float4* b;
    PCG_DEV float4 ld(uint32_t c) const { return b[(uint64_t)c << 6]; }
};
struct LdsDst {
    float4* b;
    PCG_DEV void st(uint32_t c, const float4& v) const { b[c << 6] = v; }
};
struct GlbDst {
    float4* b;
    PCG_DEV void st(uint32_t c, const float4& v) const { b[(uint64_t)c << 6] = v; }
};

struct Lane {
    uint32_t* lds;
    float* gs;
    const float4* y;
    uint32_t N, top, lane;
    SsLayout ly;
    uint32_t root = 0; // RootSrc mode of the recomputed stage top-1

    PCG_DEV uint32_t* row() const { return lds + ly.bits + lane; }
    template <typename Fn>
    PCG_DEV void with_src(uint32_t s, Fn&& f) const
    {
        if (s == top)
            f(ChanSrc{ y });
        else if (s == ly.mt)
            f(RootSrc{ y, N >> 3, row(), root });
        else if (s < ly.Sl)
            f(LdsSrc{ reinterpret_cast<const float4*>(lds) + 64u * ss_base(s) + lane });
        else
            f(GlbSrc{ reinterpret_cast<const float4*>(gs) + 64ull * (ss_base(s) - ss_base(ly.Sl)) + lane });
    }
    template <typename Fn>
    PCG_DEV void with_dst(uint32_t s, Fn&& f) const
    {
        if (s < ly.Sl)
            f(LdsDst{ reinterpret_cast<float4*>(lds) + 64u * ss_base(s) + lane });
        else
            f(GlbDst{ reinterpret_cast<float4*>(gs) + 64ull * (ss_base(s) - ss_base(ly.Sl)) + lane });
    }
    PCG_DEV uint32_t bits_at(uint32_t o, uint32_t c) const
    {
        const uint32_t w = row()[(o >> 5) << 6];
        return c >= 32 ? w : (w >> (o & 31u)) & ((1u << c) - 1u);
    }
    // positions [o, o+c) (c <= 32, inside one word) := v
    PCG_DEV void put(uint32_t o, uint32_t c, uint32_t v)
    {
        uint32_t* r = row() + ((o >> 5) << 6);
        if (c >= 32) {
            *r = v;
        } else {
            const uint32_t sh = o & 31u, msk = ((1u << c) - 1u) << sh;
            *r = (*r & ~msk) | ((v << sh) & msk);
        }
    }
    // positions [o, o+n) := the 32-bit pattern word `pat` (periodic fills), any n
    PCG_DEV void fill(uint32_t o, uint32_t n, uint32_t pat)
    {
        if (n >= 32)
            for (uint32_t q = 0; q < n / 32; ++q)
                row()[((o >> 5) + q) << 6] = pat;
        else
            put(o, n, pat);
    }
};

PCG_DEV uint32_t periodic(uint32_t pat, uint32_t period)
{
    uint32_t w = 0;
    for (uint32_t k = 0; k < 32; ++k)
        w |= ((pat >> (k % period)) & 1u) << k;
    return w;
}

// 8 lane partial sums (each lane from +0.0, chunks of 8 ascending; n < 8 padded with
// `pad`), avxconvenience.h / avx_float.h:238-250
template <typename Src>
PCG_DEV void lane_sums(const Src& src, uint32_t n, float pad, float (&s)[8])
{
#pragma unroll
    for (int j = 0; j < 8; ++j)
        s[j] = 0.0f;
    if (n < 8) { // n = 2 or 4: one unit
        const float4 v = src.ld(0);
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
            s[j] = s[j] + (j < n ? f4_at(v, j & 3u) : pad);
        return;
    }
    for (uint32_t c = 0; c < n / 4; c += 2) {
        const float4 a = src.ld(c), b = src.ld(c + 1);
        s[0] = s[0] + a.x;
        s[1] = s[1] + a.y;
        s[2] = s[2] + a.z;
        s[3] = s[3] + a.w;
        s[4] = s[4] + b.x;
        s[5] = s[5] + b.y;
        s[6] = s[6] + b.z;
        s[7] = s[7] + b.w;
    }
}
PCG_DEV float reduce8(const float (&s)[8]) { return s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7]; }

// _mm256_spc_right4_ps (avx_float.h:289-302): sign bits of the 4 outputs
PCG_DEV uint32_t spc4_bits(const float (&v)[4])
{
    float a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        a[k] = fabs_(v[k]);
    const float m = minps(minps(a[0], a[2]), minps(a[1], a[3]));
    const uint32_t par = (fbits(v[0]) ^ fbits(v[1]) ^ fbits(v[2]) ^ fbits(v[3])) >> 31;
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        o |= ((fbits(v[k]) >> 31) ^ (a[k] == m ? par : 0u)) << k;
    return o;
}

// Fast-SSC leaves (fastssc_avx_float.cpp; oracle/polar_oracle.c sc_leaf)
template <typename Src>
PCG_DEV void leaf(Lane& w, uint32_t code, const Src& src, uint32_t n, uint32_t o)
{
    switch (code) {
    case OP_L_R0:
        w.fill(o, n, 0u);
        break;
    case OP_L_R1: // bits = signs of the LLRs
        if (n < 4) {
            w.put(o, n, sgn4(src.ld(0)));
        } else {
            uint32_t acc = 0;
            for (uint32_t c = 0; c < n / 4; ++c) {
                acc |= sgn4(src.ld(c)) << ((4u * c) & 31u);
                if (n <= 32) {
                    if (4u * (c + 1) == n)
                        w.put(o, n, acc);
                } else if (((c + 1) & 7u) == 0) {
                    w.row()[((o + 4u * c) >> 5) << 6] = acc;
                    acc = 0;
                }
            }
        }
        break;
    case OP_L_REP: { // RepetitionDecoder :273-287
        float s[8];
        lane_sums(src, n, 0.0f, s);
        w.fill(o, n, (fbits(reduce8(s)) >> 31) ? 0xffffffffu : 0u);
        break;
    }
    case OP_L_DREP: { // DoubleRepetitionDecoder :303-332
        float s[8];
        lane_sums(src, n, 0.0f, s);
        float ev, od;
        if (n >= 8) {
            ev = (s[0] + s[4]) + (s[2] + s[6]);
            od = (s[1] + s[5]) + (s[3] + s[7]);
        } else {
            ev = ((s[0] + s[2]) + s[4]) + s[6];
            od = ((s[1] + s[3]) + s[5]) + s[7];
        }
        w.fill(o, n, periodic((fbits(ev) >> 31) | ((fbits(od) >> 31) << 1), 2));
        break;
    }
    case OP_L_SPC: { // SpcDecoder :342-373 (n < 8 padded with +INF)
        uint32_t par = 0, m = 0;
        float mv = __builtin_inff();
        const uint32_t nu = n < 4 ? 1u : n / 4;
        for (uint32_t c = 0; c < nu; ++c) {
            const float4 v = src.ld(c);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t i = 4u * c + k;
                if (i < n) {
                    const float x = f4_at(v, k);
                    par ^= fbits(x);
                    const float a = fabs_(x);
                    if (a < mv) {
                        mv = a;
                        m = i;
                    }
                }
            }
        }
        // padding lanes (+INF) have sign 0 and never win a strict '<'
        par >>= 31;
        if (n <= 32) {
            uint32_t acc = 0;
            for (uint32_t c = 0; c < nu; ++c)
                acc |= sgn4(src.ld(c)) << (4u * c);
            w.put(o, n, acc ^ (par << m));
        } else {
            for (uint32_t c = 0; c < n / 4; c += 8) {
                uint32_t acc = 0;
                for (uint32_t q = 0; q < 8; ++q)
                    acc |= sgn4(src.ld(c + q)) << (4u * q);
                const uint32_t base = 4u * c;
                if (m >= base && m < base + 32u)
                    acc ^= par << (m - base);
                w.row()[((o + base) >> 5) << 6] = acc;
            }
        }
        break;
    }
    case OP_L_DSPC: { // DoubleSpcDecoder :425-466 (n >= 16): per lane j running argmin, ties -> later
        float mv[8];
        uint32_t mi[8], pj[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            mv[j] = FLT_MAX_S;
            mi[j] = 0;
            pj[j] = 0;
        }
        for (uint32_t c = 0; c < n / 4; c += 2) {
            const float4 a = src.ld(c), b = src.ld(c + 1);
            const float x[8] = { a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w };
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                pj[j] ^= fbits(x[j]);
                const float av = fabs_(x[j]);
                if (!(av > mv[j])) {
                    mv[j] = av;
                    mi[j] = 4u * c + (uint32_t)j;
                }
            }
        }
        const float ce = minps(minps(mv[0], mv[4]), minps(mv[2], mv[6]));
        const float co = minps(minps(mv[1], mv[5]), minps(mv[3], mv[7]));
        uint32_t ei = 0, oi = 0;
        for (int j = 6; j >= 0; j -= 2)
            if (mv[j] == ce)
                ei = mi[j];
        for (int j = 7; j >= 1; j -= 2)
            if (mv[j] == co)
                oi = mi[j];
        const uint32_t pe = (pj[0] ^ pj[2] ^ pj[4] ^ pj[6]) >> 31, po = (pj[1] ^ pj[3] ^ pj[5] ^ pj[7]) >> 31;
        for (uint32_t c = 0; c < n / 4; c += 8) {
            const uint32_t base = 4u * c;
            const uint32_t cnt = n - base < 32u ? n - base : 32u;
            uint32_t acc = 0;
            for (uint32_t q = 0; q < cnt / 4; ++q)
                acc |= sgn4(src.ld(c + q)) << (4u * q);
            if (ei >= base && ei < base + 32u)
                acc ^= pe << (ei - base);
            if (oi >= base && oi < base + 32u)
                acc ^= po << (oi - base);
            w.put(o + base, cnt, acc);
        }
        break;
    }
    case OP_L_DSPC8: { // DoubleSpcDecoderShort8 :473-488 (multi-flip on ties)
        const float4 a = src.ld(0), b = src.ld(1);
        const float x[8] = { a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w };
        float av[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            av[j] = fabs_(x[j]);
        const float ce = minps(minps(av[0], av[4]), minps(av[2], av[6]));
        const float co = minps(minps(av[1], av[5]), minps(av[3], av[7]));
        const uint32_t pe = (fbits(x[0]) ^ fbits(x[2]) ^ fbits(x[4]) ^ fbits(x[6])) >> 31;
        const uint32_t po = (fbits(x[1]) ^ fbits(x[3]) ^ fbits(x[5]) ^ fbits(x[7])) >> 31;
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const bool ev = (j & 1) == 0;
            const uint32_t hit = av[j] == (ev ? ce : co) ? (ev ? pe : po) : 0u;
            acc |= ((fbits(x[j]) >> 31) ^ hit) << j;
        }
        w.put(o, 8, acc);
        break;
    }
    case OP_L_ZSPC8: { // ZeroSpcDecoderShort8 :556-565
        const float4 a = src.ld(0), b = src.ld(1);
        const float v[4] = { a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w };
        const uint32_t ob = spc4_bits(v);
        w.put(o, 8, ob | (ob << 4));
        break;
    }
    case OP_L_TREP: { // TripleRepetitionDecoder :572-589
        float s[8];
        lane_sums(src, n, 0.0f, s);
        const float v[4] = { s[0] + s[4], s[1] + s[5], s[2] + s[6], s[3] + s[7] };
        w.fill(o, n, periodic(spc4_bits(v), 4));
        break;
    }
    case OP_L_TYPE5:   // TypeFiveDecoder :762-792
    case OP_L_REPR1: { // RepetitionRateOneDecoderShort8 :718-739
        float l[8];
        if (code == OP_L_TYPE5) {
            lane_sums(src, n, 0.0f, l);
        } else {
            const float4 a = src.ld(0), b = src.ld(1);
            l[0] = a.x; l[1] = a.y; l[2] = a.z; l[3] = a.w;
            l[4] = b.x; l[5] = b.y; l[6] = b.z; l[7] = b.w;
        }
        float r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            r[k] = polar_f(l[k], l[k + 4]);
        const float R = (r[0] + r[1]) + (r[2] + r[3]);
        float g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            g[k] = polar_g(l[k], l[k + 4], sgn(R));
        uint32_t ob;
        if (code == OP_L_TYPE5) {
            ob = spc4_bits(g);
        } else {
            ob = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                ob |= (fbits(g[k]) >> 31) << k;
        }
        const uint32_t rb = fbits(R) >> 31;
        const uint32_t lo = ob ^ (rb ? 0xfu : 0u);
        w.fill(o, n, periodic(lo | (ob << 4), 8));
        break;
    }
    case OP_L_ZSPC: { // ZeroSpcDecoder :503-546 -- right half to both halves (Q1)
        const uint32_t h = n / 2, hq = h / 4;
        uint32_t par = 0, m = 0;
        float mv = __builtin_inff();
        for (uint32_t c = 0; c < hq; ++c) {
            const float4 l = src.ld(c), r = src.ld(c + hq);
            const float4 v = f4_add(l, r);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const float x = f4_at(v, k);
                par ^= fbits(x);
                const float a = fabs_(x);
                if (a < mv) {
                    mv = a;
                    m = 4u * c + k;
                }
            }
        }
        par >>= 31;
        for (uint32_t c = 0; c < hq; c += 8) {
            const uint32_t base = 4u * c;
            const uint32_t cnt = h - base < 32u ? h - base : 32u;
            uint32_t acc = 0;
            for (uint32_t q = 0; q < cnt / 4; ++q)
                acc |= sgn4(src.ld(hq + c + q)) << (4u * q);
            if (m >= base && m < base + 32u)
                acc ^= par << (m - base);
            w.put(o + base, cnt, acc);
            w.put(o + h + base, cnt, acc);
        }
        break;
    }
    default:
        break;
    }
}

// internal-node ops of the node at stage s (n = 2^s, h = n/2): F / G / G0 into stage s-1,
// or the fused right rate-1 of ROneNode (:205-219)
PCG_DEV void inner(Lane& w, uint32_t code, uint32_t s, uint32_t o)
{
    const uint32_t h = 1u << (s - 1);
    if (s == w.top && code != OP_RONE) { // the root's children are recomputed, never stored
        w.root = code == OP_F ? 0u : (code == OP_G ? 1u : 2u);
        return;
    }
    w.with_src(s, [&](const auto& src) {
        if (code == OP_RONE) {
            if (h < 4) { // h = 2
                const float4 d = src.ld(0);
                const uint32_t lb = w.bits_at(o, 2);
                const float r0 = polar_g(d.x, d.z, (lb & 1u) << 31), r1 = polar_g(d.y, d.w, ((lb >> 1) & 1u) << 31);
                const uint32_t rs = (fbits(r0) >> 31) | ((fbits(r1) >> 31) << 1);
                w.put(o, 4, (lb ^ rs) | (rs << 2));
            } else {
                const uint32_t hq = h / 4;
                for (uint32_t c = 0; c < hq; c += 8) {
                    const uint32_t base = 4u * c;
                    const uint32_t cnt = h - base < 32u ? h - base : 32u;
                    const uint32_t lb = w.bits_at(o + base, cnt);
                    uint32_t rs = 0;
                    for (uint32_t q = 0; q < cnt / 4; ++q)
                        rs |= sgn4(f4_g(src.ld(c + q), src.ld(c + q + hq), (lb >> (4u * q)) & 0xfu)) << (4u * q);
                    w.put(o + base, cnt, lb ^ rs);
                    w.put(o + h + base, cnt, rs);
                }
            }
            return;
        }
        w.with_dst(s - 1, [&](const auto& dst) {
            if (h < 4) { // h = 2: stage s is one unit [l0 l1 r0 r1]
                const float4 d = src.ld(0);
                float4 v;
                if (code == OP_F) {
                    v = make_float4(polar_f(d.x, d.z), polar_f(d.y, d.w), 0.0f, 0.0f);
                } else if (code == OP_G) {
                    const uint32_t lb = w.bits_at(o, 2);
                    v = make_float4(polar_g(d.x, d.z, (lb & 1u) << 31), polar_g(d.y, d.w, ((lb >> 1) & 1u) << 31),
                                    0.0f, 0.0f);
                } else {
                    v = make_float4(d.x + d.z, d.y + d.w, 0.0f, 0.0f);
                }
                dst.st(0, v);
                return;
            }
            const uint32_t hq = h / 4;
            uint32_t c = 0;
            for (; c + 4 <= hq; c += 4) { // four units in flight
                float4 av[4], bv[4];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    av[q] = src.ld(c + q);
                    bv[q] = src.ld(c + q + hq);
                }
                const uint32_t lb = code == OP_G ? w.bits_at(o + 4u * c, 16) : 0u;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    dst.st(c + q, code == OP_F ? f4_f(av[q], bv[q])
                                               : (code == OP_G ? f4_g(av[q], bv[q], (lb >> (4u * q)) & 0xfu)
                                                               : f4_add(av[q], bv[q])));
            }
            for (; c < hq; ++c) {
                const float4 a0 = src.ld(c), b0 = src.ld(c + hq);
                dst.st(c, code == OP_F ? f4_f(a0, b0)
                                       : (code == OP_G ? f4_g(a0, b0, w.bits_at(o + 4u * c, 4)) : f4_add(a0, b0)));
            }
        });
    });
}

// COMB (bit[o+i] ^= bit[o+h+i]) / COPY0 (bit[o+i] = bit[o+h+i]) on the own row
PCG_DEV void bits_op(Lane& w, uint32_t code, uint32_t s, uint32_t o)
{
    const uint32_t h = 1u << (s - 1);
    uint32_t* r = w.row();
    if (h >= 32) {
        for (uint32_t k = 0; k < h / 32; ++k) {
            const uint32_t rv = r[(((o + h) >> 5) + k) << 6];
            uint32_t& lv = r[((o >> 5) + k) << 6];
            lv = code == OP_COMB ? (lv ^ rv) : rv;
        }
    } else {
        const uint32_t sh = o & 31u, msk = ((1u << h) - 1u) << sh;
        const uint32_t x = r[(o >> 5) << 6];
        const uint32_t rr = (x >> h) & msk;
        r[(o >> 5) << 6] = code == OP_COMB ? (x ^ rr) : ((x & ~msk) | rr);
    }
}

__global__ void __launch_bounds__(64) scs_kernel(KernelArgs a, uint32_t Sl)
{
    extern __shared__ uint32_t smem_s[];
    Lane w;
    w.lds = smem_s;
    w.N = a.N;
    w.top = a.log2N;
    w.lane = threadIdx.x & 63;
    w.ly = ss_layout(a.N, Sl);
    w.gs = a.scratch + (uint64_t)blockIdx.x * w.ly.gdwords;
    const uint32_t W = a.N >= 32 ? a.N / 32 : 1u;
    const uint64_t ngroups = (a.F + 63) / 64;
    for (uint64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint64_t frame = grp * 64 + w.lane;
        const bool fok = frame < a.F;
        w.y = reinterpret_cast<const float4*>(a.llr + (fok ? frame : a.F - 1) * a.N);
        w.root = 0;
        for (uint32_t k = 0; k < a.nops; ++k) {
            const uint32_t op = ld_const(a.ops, k);
            const uint32_t code = op_code(op), s = op_stage(op), o = op_off(op);
            if (code >= OP_L_R0) {
                w.with_src(s, [&](const auto& src) { leaf(w, code, src, 1u << s, o); });
            } else if (code == OP_COMB || code == OP_COPY0) {
                bits_op(w, code, s, o);
            } else {
                inner(w, code, s, o);
            }
        }
        // output: re-encode if non-systematic, detector syndrome, info bytes
        uint32_t* r = w.row();
        if (!a.systematic) {
            for (uint32_t q = 0; q < W; ++q)
                r[q << 6] = transform_word(r[q << 6], a.N);
            for (uint32_t d = 1; d < W; d <<= 1)
                for (uint32_t q = 0; q < W; ++q)
                    if (!(q & d))
                        r[q << 6] ^= r[(q + d) << 6];
        }
        uint32_t syn = a.crc_c0;
        for (uint32_t rb = 0; rb < a.crc_bits; ++rb) {
            uint32_t pc = 0;
            for (uint32_t q = 0; q < W; ++q)
                pc += __builtin_popcount(r[q << 6] & a.crc_rows[rb * W + q]);
            syn ^= (pc & 1u) << rb;
        }
        if (fok) {
            uint8_t* out = a.info + frame * a.kb;
            uint32_t cw = 0xffffffffu, word = 0;
            for (uint32_t b = 0; b < a.kb; ++b) {
                uint32_t byte = 0;
                for (uint32_t q = 0; q < 8; ++q) {
                    const uint32_t idx = 8 * b + q;
                    if (idx < a.K) {
                        const uint32_t pos = a.info_pos[idx];
                        if ((pos >> 5) != cw) {
                            cw = pos >> 5;
                            word = r[cw << 6];
                        }
                        byte |= ((word >> (pos & 31u)) & 1u) << (7 - q);
                    }
                }
                out[b] = (uint8_t)byte;
            }
            if (a.ok)
                a.ok[frame] = syn == 0 ? 1 : 0;
        }
    }
}

int resident(uint32_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scs_kernel, 64, lds_bytes) != hipSuccess)
        n = 0;
    return n;
}

} // namespace

// LDS / scratch layout of the lane-serial Fast-SSC kernel: stages < Sl in LDS within
// PCG_SCS_LDS_KB (default 40 KB: stages < 7 in LDS, 4 waves/CU at N = 1024 -- measured
// 6.8e7 cw/s at 12 KB / 12 waves, 7.7e7 at 40 KB / 4 waves, 5.0e7 all-LDS / 1 wave).
int scs_layout(uint32_t N, uint32_t* lds_dwords, uint32_t* Sl, uint64_t* scratch_dwords)
{
    if (N < 8)
        return -4;
    uint32_t budget = 40u * 1024u;
    if (const char* e = getenv("PCG_SCS_LDS_KB"))
        budget = (uint32_t)atoi(e) * 1024u;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    uint32_t best = 1;
    for (uint32_t s = 1; s <= top - 1; ++s)
        if (ss_layout(N, s).lds * 4u <= budget)
            best = s;
    if (const char* e = getenv("PCG_SCS_SL")) { // dev override, ignored when out of range
        const uint32_t v = (uint32_t)atoi(e);
        if (v >= 1 && v <= top - 1)
            best = v;
    }
    const SsLayout y = ss_layout(N, best);
    if (y.lds * 4u > 160u * 1024u)
        return -4;
    *lds_dwords = y.lds;
    *Sl = y.Sl;
    *scratch_dwords = y.gdwords;
    return 0;
}

uint64_t scs_wave_cap(uint32_t lds_dwords)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int res = resident(lds_dwords * 4u);
    uint64_t wpc = res > 0 ? (uint64_t)res : 1;
    if (wpc > 16)
        wpc = 16;
    wpc = env_wpc("PCG_SCS_WPC", wpc);
    if (getenv("PCG_DEBUG_OCC"))
        fprintf(stderr, "[pcg] scs: lds %u B, resident %d waves/CU, using %llu\n", lds_dwords * 4u, res,
                (unsigned long long)wpc);
    return (uint64_t)cus * wpc;
}

int launch_scs(const KernelArgs& a, hipStream_t stream)
{
    const uint64_t grid = a.units;
    if (grid == 0) // no waves for a non-empty batch: an error, never a silent no-op
        return a.F ? -4 : 0;
    hipLaunchKernelGGL(scs_kernel, dim3((uint32_t)grid), dim3(64), (size_t)a.wave_lds_floats * 4u, stream, a,
                       a.lds_stage_limit);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

} // namespace pcg
