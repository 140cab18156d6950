// scq_kernel.hip -- LDS-resident batched Fast-SSC ("SC") polar decoding on CDNA4 (gfx950).
//
// Q lanes per codeword, G = 64 / Q codewords per wave.  Each codeword keeps its whole
// decoder state in LDS: the LLR stages 1 <= s < log2 N (stage s at float offset 2^s, so
// the root's children are stored, not recomputed) and the codeword estimate as packed
// sign bits.  The channel frame is read from HBM exactly twice per codeword -- once by
// the root's F (left child), once by its G (right child), both coalesced float4 rows
// (Q lanes x 16 B contiguous) -- so the kernel moves ~2 x 4N bytes where the lane-serial
// scs_kernel.hip, whose per-wave state (64 codewords) must spill to a global slab,
// moves ~16x the algorithmic bytes (profiles/r02b_bench_sc.json).
//
// The wave walks the plan's Fast-SSC schedule (plan.cpp sc_emit, the reference's
// FastSscAvx tree in decode order) uniformly.  F / G / G0 / fused ROne, Rate-0, Rate-1,
// Repetition and SPC leaves run across the Q lanes of a codeword (float4 chunks, packed
// words assembled with DPP); the remaining leaf kinds run on the codeword's first lane
// with the reference's scalar loops (oracle/polar_oracle.c sc_leaf), as scs_kernel.hip
// does for every leaf.  Every arithmetic step keeps the AVX2 reference's lane order and
// sign-of-zero behaviour (fastssc_avx_float.cpp).
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"

#ifndef PCG_RTC
#include <stdio.h>
#include <stdlib.h>
#endif

namespace pcg {

namespace {

constexpr float FLT_MAX_Q = 3.40282347e+38f;

// per-codeword LDS region: alpha floats (stage s at 2^s; stages < log2 N, or < log2 N - 1
// when the root's children are recomputed from the channel, V), bit words, pad
constexpr __host__ __device__ inline uint32_t scq_words(uint32_t N) { return N >= 32 ? N / 32 : 1u; }
constexpr __host__ __device__ inline uint32_t scq_alpha(uint32_t N, bool V) { return V ? N / 2 : N; }
constexpr __host__ __device__ inline uint32_t scq_region(uint32_t N, bool V)
{
    // + 4 dwords so that codeword regions of one wave start on different LDS banks
    return ((scq_alpha(N, V) + scq_words(N) + 3u) & ~3u) + 4u;
}

PCG_DEV float4 q_f(const float4& a, const float4& b)
{
    return make_float4(polar_f(a.x, b.x), polar_f(a.y, b.y), polar_f(a.z, b.z), polar_f(a.w, b.w));
}
// G of 4 elements with their bits at positions k0 .. k0+3 of nib (k0 + 3 < 32)
PCG_DEV float4 q_g(const float4& a, const float4& b, uint32_t nib, uint32_t k0 = 0)
{
    return make_float4(polar_g_bit(a.x, b.x, nib, k0), polar_g_bit(a.y, b.y, nib, k0 + 1),
                       polar_g_bit(a.z, b.z, nib, k0 + 2), polar_g_bit(a.w, b.w, nib, k0 + 3));
}
PCG_DEV float4 q_add(const float4& a, const float4& b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
PCG_DEV uint32_t q_sgn4(const float4& v)
{
    return (fbits(v.x) >> 31) | ((fbits(v.y) >> 31) << 1) | ((fbits(v.z) >> 31) << 2) | ((fbits(v.w) >> 31) << 3);
}
PCG_DEV float q_at(const float4& v, uint32_t k) { return k == 0 ? v.x : (k == 1 ? v.y : (k == 2 ? v.z : v.w)); }

// Lane J of this lane's codeword group.  Q = 16: the group is one DPP row, so the broadcast
// is a row_newbcast move (VALU, no LDS crossbar round trip); other Q: ds_bpermute.
template <int Q, int J>
PCG_DEV uint32_t gbc(uint32_t v, int base)
{
    if constexpr (Q == 16)
        return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + J, 0xF, 0xF, false);
    else
        return (uint32_t)__shfl((int)v, base + J, 64);
}
// o[j] = lane j of the group, j < N
template <int Q, int N, int J = 0>
PCG_DEV void gbc_all(uint32_t v, int base, uint32_t (&o)[N])
{
    if constexpr (J < N) {
        o[J] = gbc<Q, J>(v, base);
        gbc_all<Q, N, J + 1>(v, base, o);
    }
}
template <int Q, int N>
PCG_DEV void gbc_allf(float v, int base, float (&o)[N])
{
    uint32_t u[N];
    gbc_all<Q, N>(fbits(v), base, u);
#pragma unroll
    for (int j = 0; j < N; ++j)
        o[j] = ubits(u[j]);
}
// lane i ^ 8 of the group (Q = 16: row_ror:8)
template <int Q>
PCG_DEV float gxor8(float v, int base, uint32_t i)
{
    if constexpr (Q == 16)
        return ubits((uint32_t)__builtin_amdgcn_update_dpp(0, (int)fbits(v), 0x128, 0xF, 0xF, false));
    else
        return __shfl(v, base + (int)(i ^ 8u), 64);
}

// OR of a value over aligned groups of 8 lanes (exact xor partners 1, 2, 4)
PCG_DEV uint32_t or8(uint32_t v)
{
    v |= xpartner<1>(v);
    v |= xpartner<2>(v);
    v |= xpartner<4>(v);
    return v;
}

// A stage buffer: LDS floats of this codeword, its channel frame (root stage), or -- V
// kernels -- a child of the root recomputed from the channel wherever it is read: F(y_i,
// y_i+N/2) (mode 1), G(y_i, y_i+N/2, bit_i) with the codeword's left-half bits (mode 2),
// y_i + y_i+N/2 below a ZeroRNode root (mode 3).  The mode is wave-uniform.
// Two source types, so that code reading the stored stages never carries the recompute
// path (register pressure): PSrc (LDS stage or channel frame), VSrc (recomputed child).
struct PSrc {
    const float* p;
    PCG_DEV float4 ld(uint32_t c) const { return reinterpret_cast<const float4*>(p)[c]; }
    PCG_DEV float at(uint32_t i) const { return p[i]; }
};
struct VSrc {
    const float* y;
    const uint32_t* row;
    uint32_t half;
    uint32_t mode;
    PCG_DEV float4 ld(uint32_t c) const
    {
        const float4 a = reinterpret_cast<const float4*>(y)[c], b = reinterpret_cast<const float4*>(y + half)[c];
        if (mode == 1)
            return q_f(a, b);
        if (mode == 3)
            return q_add(a, b);
        return q_g(a, b, row[c >> 3], (4u * c) & 31u);
    }
    PCG_DEV float at(uint32_t i) const
    {
        const float a = y[i], b = y[i + half];
        if (mode == 1)
            return polar_f(a, b);
        if (mode == 3)
            return a + b;
        return polar_g_bit(a, b, row[i >> 5], i & 31u);
    }
};

template <int Q>
struct Cw {
    float* alpha;   // this codeword's LDS region
    uint32_t* row;  // its packed bit words
    const float* y; // its channel frame
    uint32_t sub;   // lane within the codeword's group
    uint32_t N, top;
    uint32_t virt;  // 1: the root's children are recomputed (Src modes 1-3), never stored
    uint32_t root;  // Src mode of the recomputed children

    // stage s as a source: f(PSrc) for stored stages and the channel, f(VSrc) for a
    // recomputed child of the root
    PCG_DEV PSrc psrc(uint32_t s) const { return PSrc{ s == top ? y : alpha + (1u << s) }; }
    template <typename Fn>
    PCG_DEV void with_src(uint32_t s, Fn&& f) const
    {
        if (virt && s == top - 1)
            f(VSrc{ y, row, N / 2, root });
        else
            f(PSrc{ s == top ? y : alpha + (1u << s) });
    }
    PCG_DEV uint32_t nib(uint32_t pos) const { return (row[pos >> 5] >> (pos & 31u)) & 0xfu; }
    // positions [o, o+c) (c <= 32, inside one word) := v      (single lane)
    PCG_DEV void put(uint32_t o, uint32_t c, uint32_t v) const
    {
        uint32_t* r = row + (o >> 5);
        if (c >= 32) {
            *r = v;
        } else {
            const uint32_t sh = o & 31u, msk = ((1u << c) - 1u) << sh;
            *r = (*r & ~msk) | ((v << sh) & msk);
        }
    }
    // positions [o, o+n) := periodic 32-bit pattern `pat`     (group-parallel)
    PCG_DEV void fill(uint32_t o, uint32_t n, uint32_t pat) const
    {
        if (n >= 32) {
            for (uint32_t q = sub; q < n / 32; q += Q)
                row[(o >> 5) + q] = pat;
        } else if (sub == 0) {
            put(o, n, pat);
        }
    }
    // chunk-parallel nibbles -> packed bits of [o, o + 4*nc): lanes hold the nibble of
    // chunk c = sub + t*Q in `v`; every lane of the group calls this with the same t
    PCG_DEV void store_nibbles(uint32_t o, uint32_t nc, uint32_t t, uint32_t v) const
    {
        const uint32_t c = sub + t * Q;
        const uint32_t w = or8(c < nc ? v << (4u * (c & 7u)) : 0u);
        if (nc >= 8) {
            if ((c & 7u) == 0 && c < nc)
                row[(o >> 5) + (c >> 3)] = w;
        } else if (sub == 0) {
            put(o, 4u * nc, w);
        }
    }
};

PCG_DEV uint32_t periodic_q(uint32_t pat, uint32_t period)
{
    uint32_t w = 0;
    for (uint32_t k = 0; k < 32; ++k)
        w |= ((pat >> (k % period)) & 1u) << k;
    return w;
}

// _mm256_spc_right4_ps (avx_float.h:289-302): sign bits of the 4 outputs
PCG_DEV uint32_t spc4_q(const float (&v)[4])
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

// 8 lane partial sums of the reference (lanes from +0.0, chunks of 8 ascending; n < 8
// padded with +0.0), serial on one lane (avxconvenience.h:256-272, avx_float.h:238-250)
template <typename SRC>
PCG_DEV void lane_sums_q(const SRC& src, uint32_t n, float (&s)[8])
{
#pragma unroll
    for (int j = 0; j < 8; ++j)
        s[j] = 0.0f;
    if (n < 8) {
        for (uint32_t j = 0; j < 8; ++j)
            s[j] = s[j] + (j < n ? src.at(j) : 0.0f);
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

// Leaf kinds run on the group's first lane with the reference's scalar loops
// (fastssc_avx_float.cpp:303-792, oracle/polar_oracle.c sc_leaf).
template <int Q, typename SRC>
PCG_DEV void serial_leaf(const Cw<Q>& w, uint32_t code, const SRC& src, uint32_t n, uint32_t o)
{
    switch (code) {
    case OP_L_REP: { // n < 8 (larger repetition leaves run group-parallel)
        float s[8];
        lane_sums_q(src, n, s);
        const float S = s[0] + s[1] + s[2] + s[3] + s[4] + s[5] + s[6] + s[7];
        w.put(o, n, (fbits(S) >> 31) ? 0xffffffffu : 0u);
        break;
    }
    case OP_L_SPC: { // n < 8, padded with +INF (never wins a strict '<', sign 0)
        uint32_t par = 0, m = 0, acc = 0;
        float mv = __builtin_inff();
        for (uint32_t i = 0; i < n; ++i) {
            const float x = src.at(i);
            par ^= fbits(x);
            acc |= (fbits(x) >> 31) << i;
            const float a = fabs_(x);
            if (a < mv) {
                mv = a;
                m = i;
            }
        }
        w.put(o, n, acc ^ ((par >> 31) << m));
        break;
    }
    case OP_L_R1: // n < 4
    {
        uint32_t acc = 0;
        for (uint32_t i = 0; i < n; ++i)
            acc |= (fbits(src.at(i)) >> 31) << i;
        w.put(o, n, acc);
        break;
    }
    case OP_L_DREP: { // DoubleRepetitionDecoder :303-332
        float s[8];
        lane_sums_q(src, n, s);
        float ev, od;
        if (n >= 8) {
            ev = (s[0] + s[4]) + (s[2] + s[6]);
            od = (s[1] + s[5]) + (s[3] + s[7]);
        } else {
            ev = ((s[0] + s[2]) + s[4]) + s[6];
            od = ((s[1] + s[3]) + s[5]) + s[7];
        }
        const uint32_t pat = periodic_q((fbits(ev) >> 31) | ((fbits(od) >> 31) << 1), 2);
        if (n >= 32)
            for (uint32_t q = 0; q < n / 32; ++q)
                w.row[(o >> 5) + q] = pat;
        else
            w.put(o, n, pat);
        break;
    }
    case OP_L_DSPC: { // DoubleSpcDecoder :425-466 (n >= 16): per AVX lane running argmin, ties -> later
        float mv[8];
        uint32_t mi[8], pj[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            mv[j] = FLT_MAX_Q;
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
                acc |= q_sgn4(src.ld(c + q)) << (4u * q);
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
        const uint32_t ob = spc4_q(v);
        w.put(o, 8, ob | (ob << 4));
        break;
    }
    case OP_L_TREP: { // TripleRepetitionDecoder :572-589
        float s[8];
        lane_sums_q(src, n, s);
        const float v[4] = { s[0] + s[4], s[1] + s[5], s[2] + s[6], s[3] + s[7] };
        const uint32_t pat = periodic_q(spc4_q(v), 4);
        for (uint32_t q = 0; q < n / 32; ++q)
            w.row[(o >> 5) + q] = pat;
        if (n < 32)
            w.put(o, n, pat);
        break;
    }
    case OP_L_TYPE5:   // TypeFiveDecoder :762-792
    case OP_L_REPR1: { // RepetitionRateOneDecoderShort8 :718-739
        float l[8];
        if (code == OP_L_TYPE5) {
            lane_sums_q(src, n, l);
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
            ob = spc4_q(g);
        } else {
            ob = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                ob |= (fbits(g[k]) >> 31) << k;
        }
        const uint32_t lo = ob ^ ((fbits(R) >> 31) ? 0xfu : 0u);
        const uint32_t pat = periodic_q(lo | (ob << 4), 8);
        for (uint32_t q = 0; q < n / 32; ++q)
            w.row[(o >> 5) + q] = pat;
        if (n < 32)
            w.put(o, n, pat);
        break;
    }
    case OP_L_ZSPC: { // ZeroSpcDecoder :503-546 -- right half to both halves (Q1)
        const uint32_t h = n / 2, hq = h / 4;
        uint32_t par = 0, m = 0;
        float mv = __builtin_inff();
        for (uint32_t c = 0; c < hq; ++c) {
            const float4 v = q_add(src.ld(c), src.ld(c + hq));
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const float x = q_at(v, k);
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
                acc |= q_sgn4(src.ld(hq + c + q)) << (4u * q);
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

// The reference's 8 AVX lane sums s_j (each from +0.0, chunks of 8 ascending; n < 8
// padded with +0.0): group lane j < 8 accumulates s_j in the reference's order, then every
// lane of the group receives all eight.
template <int Q, typename SRC>
PCG_DEV void grp_lane_sums(const Cw<Q>& w, const SRC& src, uint32_t n, float (&s)[8])
{
    float acc = 0.0f;
    if (w.sub < 8) {
        if (n < 8)
            acc = acc + (w.sub < n ? src.at(w.sub) : 0.0f);
        else
            for (uint32_t i = w.sub; i < n; i += 8)
                acc = acc + src.at(i);
    }
    const int base = (int)(__lane_id() & ~(uint32_t)(Q - 1));
    gbc_allf<Q, 8>(acc, base, s);
}

// positions [o, o+n) := periodic pattern, every lane holding the same `pat`
template <int Q>
PCG_DEV void fill_any(const Cw<Q>& w, uint32_t o, uint32_t n, uint32_t pat)
{
    w.fill(o, n, pat);
}

// Leaf kinds whose reductions follow the 8 AVX lanes, run on the group (the reference's
// loops per AVX lane on group lanes 0..7; the tail math, identical in every lane)
template <int Q, typename SRC>
PCG_DEV bool grp_leaf(const Cw<Q>& w, uint32_t code, const SRC& src, uint32_t n, uint32_t o)
{
    switch (code) {
    case OP_L_DREP: { // DoubleRepetitionDecoder :303-332
        float s[8];
        grp_lane_sums(w, src, n, s);
        float ev, od;
        if (n >= 8) {
            ev = (s[0] + s[4]) + (s[2] + s[6]);
            od = (s[1] + s[5]) + (s[3] + s[7]);
        } else {
            ev = ((s[0] + s[2]) + s[4]) + s[6];
            od = ((s[1] + s[3]) + s[5]) + s[7];
        }
        fill_any(w, o, n, periodic_q((fbits(ev) >> 31) | ((fbits(od) >> 31) << 1), 2));
        return true;
    }
    case OP_L_TREP: { // TripleRepetitionDecoder :572-589
        float s[8];
        grp_lane_sums(w, src, n, s);
        const float v[4] = { s[0] + s[4], s[1] + s[5], s[2] + s[6], s[3] + s[7] };
        fill_any(w, o, n, periodic_q(spc4_q(v), 4));
        return true;
    }
    case OP_L_TYPE5:   // TypeFiveDecoder :762-792
    case OP_L_REPR1: { // RepetitionRateOneDecoderShort8 :718-739
        float l[8];
        if (code == OP_L_TYPE5) {
            grp_lane_sums(w, src, n, l);
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
            ob = spc4_q(g);
        } else {
            ob = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                ob |= (fbits(g[k]) >> 31) << k;
        }
        const uint32_t lo = ob ^ ((fbits(R) >> 31) ? 0xfu : 0u);
        fill_any(w, o, n, periodic_q(lo | (ob << 4), 8));
        return true;
    }
    case OP_L_DSPC: { // DoubleSpcDecoder :425-466 (n >= 16): AVX lane j's running argmin (ties
                      // -> later index) and parity on group lane j, then the reference's combine
        float mvj = FLT_MAX_Q;
        uint32_t mij = 0, pjj = 0;
        if (w.sub < 8)
            for (uint32_t i = w.sub; i < n; i += 8) {
                const float x = src.at(i);
                pjj ^= fbits(x);
                const float av = fabs_(x);
                if (!(av > mvj)) {
                    mvj = av;
                    mij = i;
                }
            }
        const int base = (int)(__lane_id() & ~(uint32_t)(Q - 1));
        float mv[8];
        uint32_t mi[8], pjs[8];
        uint32_t pe = 0, po = 0;
        gbc_allf<Q, 8>(mvj, base, mv);
        gbc_all<Q, 8>(mij, base, mi);
        gbc_all<Q, 8>(pjj, base, pjs);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t pj = pjs[j];
            if (j & 1)
                po ^= pj;
            else
                pe ^= pj;
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
        pe >>= 31;
        po >>= 31;
        const uint32_t nc = n / 4;
        for (uint32_t t = 0; t * Q < nc; ++t) {
            const uint32_t c = w.sub + t * Q;
            uint32_t v = c < nc ? q_sgn4(src.ld(c)) : 0u;
            if ((ei >> 2) == c)
                v ^= pe << (ei & 3u);
            if ((oi >> 2) == c)
                v ^= po << (oi & 3u);
            w.store_nibbles(o, nc, t, v);
        }
        return true;
    }
    case OP_L_ZSPC: { // ZeroSpcDecoder :503-546 -- right half to both halves (Q1)
        const uint32_t h = n / 2, hq = h / 4;
        if (hq < 2)
            return false;
        float mv = __builtin_inff();
        uint32_t mi = 0xffffffffu, par = 0;
        for (uint32_t c = w.sub; c < hq; c += Q) {
            const float4 v = q_add(src.ld(c), src.ld(c + hq));
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const float x = q_at(v, k);
                par ^= fbits(x);
                const float a = fabs_(x);
                if (a < mv) {
                    mv = a;
                    mi = 4u * c + k;
                }
            }
        }
        grp_argmin(mv, mi, Q);
        par = grp_xor(par, Q) >> 31;
        if (mi == 0xffffffffu)
            mi = 0;
        for (uint32_t t = 0; t * Q < hq; ++t) {
            const uint32_t c = w.sub + t * Q;
            uint32_t v = c < hq ? q_sgn4(src.ld(hq + c)) : 0u;
            if ((mi >> 2) == c)
                v ^= par << (mi & 3u);
            w.store_nibbles(o, hq, t, v);
            w.store_nibbles(o + h, hq, t, v);
        }
        return true;
    }
    default:
        return false;
    }
}

template <int Q, typename SRC>
PCG_DEV void leaf_body(const Cw<Q>& w, uint32_t code, const SRC& src, uint32_t s, uint32_t o)
{
    const uint32_t n = 1u << s;
    if (code == OP_L_R0) { // RateZeroDecoder: +INF bits
        w.fill(o, n, 0u);
        return;
    }
    if (code == OP_L_R1 && n >= 4) { // RateOneDecoder: bits = signs
        const uint32_t nc = n / 4;
        for (uint32_t t = 0; t * Q < nc; ++t) {
            const uint32_t c = w.sub + t * Q;
            w.store_nibbles(o, nc, t, c < nc ? q_sgn4(src.ld(c)) : 0u);
        }
        return;
    }
    if (code == OP_L_REP && n >= 8) { // RepetitionDecoder :273-287, AVX lane j on group lane j
        float acc = 0.0f;
        if (w.sub < 8)
            for (uint32_t i = w.sub; i < n; i += 8)
                acc = acc + src.at(i);
        const uint32_t base = __lane_id() & ~(uint32_t)(Q - 1);
        float t[8];
        gbc_allf<Q, 8>(acc, (int)base, t);
        float S = t[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)
            S = S + t[j];
        w.fill(o, n, (fbits(S) >> 31) ? 0xffffffffu : 0u);
        return;
    }
    if (code == OP_L_SPC && n >= 8) { // SpcDecoder :342-373: argmin |x| (lowest index), parity
        const uint32_t nc = n / 4;
        float mv = __builtin_inff();
        uint32_t mi = 0xffffffffu, par = 0;
        for (uint32_t c = w.sub; c < nc; c += Q) {
            const float4 v = src.ld(c);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) {
                const float x = q_at(v, k);
                par ^= fbits(x);
                const float a = fabs_(x);
                if (a < mv) {
                    mv = a;
                    mi = 4u * c + k;
                }
            }
        }
        grp_argmin(mv, mi, Q);
        par = grp_xor(par, Q) >> 31;
        if (mi == 0xffffffffu)
            mi = 0;
        for (uint32_t t = 0; t * Q < nc; ++t) {
            const uint32_t c = w.sub + t * Q;
            uint32_t v = c < nc ? q_sgn4(src.ld(c)) : 0u;
            if ((mi >> 2) == c)
                v ^= par << (mi & 3u);
            w.store_nibbles(o, nc, t, v);
        }
        return;
    }
    if (grp_leaf<Q>(w, code, src, n, o))
        return;
    if (w.sub == 0)
        serial_leaf<Q>(w, code, src, n, o);
}

// (leaves never read a recomputed child: the host stores the children of a root with a
// leaf child, capi.cpp)
template <int Q>
PCG_DEV void leaf_q(const Cw<Q>& w, uint32_t code, uint32_t s, uint32_t o)
{
    leaf_body<Q>(w, code, w.psrc(s), s, o);
}

// A size-8 Fast-SSC leaf on 8 LLRs in registers: the 8 output sign bits (bit i = position i).
// Exactly the reference's n = 8 arithmetic (lane sums of one chunk are +0.0 + x_j).
PCG_DEV uint32_t leaf8_bits(uint32_t code, const float (&x)[8])
{
    uint32_t sg = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        sg |= (fbits(x[j]) >> 31) << j;
    switch (code) {
    case OP_L_R0:
        return 0u;
    case OP_L_R1:
        return sg;
    case OP_L_REP: { // :273-287
        float S = 0.0f + x[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)
            S = S + (0.0f + x[j]);
        return (fbits(S) >> 31) ? 0xffu : 0u;
    }
    case OP_L_SPC: { // :342-373, n = 8: argmin lowest index, parity of all signs
        uint32_t par = 0, m = 0;
        float mv = __builtin_inff();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            par ^= fbits(x[j]);
            const float a = fabs_(x[j]);
            if (a < mv) {
                mv = a;
                m = (uint32_t)j;
            }
        }
        return sg ^ ((par >> 31) << m);
    }
    case OP_L_DREP: { // :303-332, n = 8
        const float ev = ((0.0f + x[0]) + (0.0f + x[4])) + ((0.0f + x[2]) + (0.0f + x[6]));
        const float od = ((0.0f + x[1]) + (0.0f + x[5])) + ((0.0f + x[3]) + (0.0f + x[7]));
        const uint32_t e = fbits(ev) >> 31, d = fbits(od) >> 31;
        return (e ? 0x55u : 0u) | (d ? 0xaau : 0u);
    }
    case OP_L_DSPC8: { // :473-488 (multi-flip on ties)
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
        return acc;
    }
    case OP_L_ZSPC8: { // :556-565
        const float v[4] = { x[0] + x[4], x[1] + x[5], x[2] + x[6], x[3] + x[7] };
        const uint32_t ob = spc4_q(v);
        return ob | (ob << 4);
    }
    case OP_L_TYPE5:   // :762-792, n = 8 (lane sums of one chunk)
    case OP_L_REPR1: { // :718-739
        float l[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            l[j] = code == OP_L_TYPE5 ? 0.0f + x[j] : x[j];
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
            ob = spc4_q(g);
        } else {
            ob = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                ob |= (fbits(g[k]) >> 31) << k;
        }
        return (ob ^ ((fbits(R) >> 31) ? 0xfu : 0u)) | (ob << 4);
    }
    default:
        return 0u;
    }
}

// A size-16 Fast-SSC leaf on 16 LLRs in registers: the 16 output sign bits.  The reference's
// n = 16 arithmetic: AVX lane sums s_j = (+0.0 + x_j) + x_(8+j) (fastssc_avx_float.cpp:273-792).
PCG_DEV uint32_t leaf16_bits(uint32_t code, const float (&x)[16])
{
    uint32_t sg = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
        sg |= (fbits(x[j]) >> 31) << j;
    float s[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        s[j] = (0.0f + x[j]) + x[8 + j];
    switch (code) {
    case OP_L_R0:
        return 0u;
    case OP_L_R1:
        return sg;
    case OP_L_REP: { // :273-287
        float S = s[0];
#pragma unroll
        for (int j = 1; j < 8; ++j)
            S = S + s[j];
        return (fbits(S) >> 31) ? 0xffffu : 0u;
    }
    case OP_L_SPC: { // :342-373: argmin lowest index, parity of all signs
        uint32_t par = 0, m = 0;
        float mv = __builtin_inff();
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            par ^= fbits(x[j]);
            const float a = fabs_(x[j]);
            if (a < mv) {
                mv = a;
                m = (uint32_t)j;
            }
        }
        return sg ^ ((par >> 31) << m);
    }
    case OP_L_DREP: { // :303-332
        const float ev = (s[0] + s[4]) + (s[2] + s[6]);
        const float od = (s[1] + s[5]) + (s[3] + s[7]);
        return ((fbits(ev) >> 31) ? 0x5555u : 0u) | ((fbits(od) >> 31) ? 0xaaaau : 0u);
    }
    case OP_L_DSPC: { // :425-466: AVX lane j's running argmin (ties -> later index), parities
        float mv[8];
        uint32_t mi[8];
        uint32_t pe = 0, po = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            mv[j] = FLT_MAX_Q;
            mi[j] = 0;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const float v = x[8 * k + j];
                if (j & 1)
                    po ^= fbits(v);
                else
                    pe ^= fbits(v);
                const float av = fabs_(v);
                if (!(av > mv[j])) {
                    mv[j] = av;
                    mi[j] = (uint32_t)(8 * k + j);
                }
            }
        }
        const float ce = minps(minps(mv[0], mv[4]), minps(mv[2], mv[6]));
        const float co = minps(minps(mv[1], mv[5]), minps(mv[3], mv[7]));
        uint32_t ei = 0, oi = 0;
#pragma unroll
        for (int j = 6; j >= 0; j -= 2)
            if (mv[j] == ce)
                ei = mi[j];
#pragma unroll
        for (int j = 7; j >= 1; j -= 2)
            if (mv[j] == co)
                oi = mi[j];
        return sg ^ ((pe >> 31) << ei) ^ ((po >> 31) << oi);
    }
    case OP_L_TREP: { // :572-589
        const float v[4] = { s[0] + s[4], s[1] + s[5], s[2] + s[6], s[3] + s[7] };
        const uint32_t ob = spc4_q(v);
        return ob | (ob << 4) | (ob << 8) | (ob << 12);
    }
    case OP_L_TYPE5: { // :762-792
        float r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            r[k] = polar_f(s[k], s[k + 4]);
        const float R = (r[0] + r[1]) + (r[2] + r[3]);
        float g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            g[k] = polar_g(s[k], s[k + 4], sgn(R));
        const uint32_t ob = spc4_q(g);
        const uint32_t p8 = (ob ^ ((fbits(R) >> 31) ? 0xfu : 0u)) | (ob << 4);
        return p8 | (p8 << 8);
    }
    case OP_L_ZSPC: { // :503-546 -- right half to both halves (Q1)
        uint32_t par = 0, m = 0, rs = 0;
        float mv = __builtin_inff();
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float v = x[i] + x[8 + i];
            par ^= fbits(v);
            rs |= (fbits(x[8 + i]) >> 31) << i;
            const float a = fabs_(v);
            if (a < mv) {
                mv = a;
                m = (uint32_t)i;
            }
        }
        const uint32_t hb = rs ^ ((par >> 31) << m);
        return hb | (hb << 8);
    }
    default:
        return 0u;
    }
}

// OP_Q16 / OP_Q16R: a size-16 node over size-8 leaves in registers on the codeword's first
// lane -- RateRNode (:148-155: F, left leaf, G, right leaf, Combine) or ROneNode
// (:198-219: F, left leaf, fused right rate-1).  16 LLRs in, 16 bits out.
// (a = the node's LLRs 0..7, b = 8..15; right = ROne node)
template <int Q>
PCG_DEV void q16_core(const Cw<Q>& w, const float (&a)[8], const float (&b)[8], bool rone, uint32_t o,
                      uint32_t desc)
{
    float l[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        l[i] = polar_f(a[i], b[i]);
    const uint32_t bl = leaf8_bits(desc & 0xffu, l);
    float r[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        r[i] = polar_g_bit(a[i], b[i], bl, (uint32_t)i);
    uint32_t br;
    if (!rone) {
        br = leaf8_bits((desc >> 8) & 0xffu, r);
    } else { // right rate-1: bits = signs of r; left := left ^ right
        br = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            br |= (fbits(r[i]) >> 31) << i;
    }
    w.put(o, 16, (bl ^ br) | (br << 8));
}

template <int Q, typename SRC>
PCG_DEV void q16_body(const Cw<Q>& w, const SRC& src, uint32_t code, uint32_t o, uint32_t desc)
{
    const float4 c0 = src.ld(0), c1 = src.ld(1), c2 = src.ld(2), c3 = src.ld(3);
    const float a[8] = { c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w };
    const float b[8] = { c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w };
    q16_core<Q>(w, a, b, code == OP_Q16R, o, desc);
}

// OP_Q16F / OP_Q16G: the size-32 parent's F (left child) or G (right child, with the
// parent's left-half bits) from its 32 LLRs, then the child as in q16_core.
template <int Q>
PCG_DEV void q16x(const Cw<Q>& w, uint32_t code, uint32_t o, uint32_t desc)
{
    if (w.sub != 0)
        return;
    const bool right = code == OP_Q16G;
    const uint32_t op = right ? o - 16u : o; // the parent's offset
    const PSrc src = w.psrc(5);
    float4 v[8];
#pragma unroll
    for (uint32_t c = 0; c < 8; ++c)
        v[c] = src.ld(c);
    const uint32_t lb = right ? (w.row[op >> 5] >> (op & 31u)) : 0u; // bits op .. op+15
    float x[16];
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const float p0 = q_at(v[i >> 2], i & 3u), p1 = q_at(v[4 + (i >> 2)], i & 3u);
        x[i] = right ? polar_g_bit(p0, p1, lb, i) : polar_f(p0, p1);
    }
    if ((desc >> 17) & 1u) { // the child is a size-16 leaf (code in the low byte)
        w.put(o, 16, leaf16_bits(desc & 0xffu, x));
        return;
    }
    float a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = x[i];
        b[i] = x[i + 8];
    }
    q16_core<Q>(w, a, b, (desc >> 16) & 1u, o, desc);
}

// The fused size-16 ops across the codeword's group (Q >= 16): element i of the size-16
// node on group lane i (the elementwise F / G in one instruction each), the size-8 leaves
// on the eight values broadcast to every lane (the same arithmetic as q16_core / q16x, so
// the same bits), lane 0 storing.
template <int Q>
PCG_DEV void q16_par(const Cw<Q>& w, uint32_t code, uint32_t o, uint32_t desc)
{
    const uint32_t i = w.sub & 15u;
    const int base = (int)(__lane_id() & ~(uint32_t)(Q - 1));
    float x;
    if (code == OP_Q16F || code == OP_Q16G) {
        const bool right = code == OP_Q16G;
        const uint32_t op = right ? o - 16u : o; // the parent's offset
        const PSrc src = w.psrc(5);
        const float p0 = src.at(i), p1 = src.at(i + 16);
        const uint32_t lb = right ? ((w.row[op >> 5] >> (op & 31u)) >> i) & 1u : 0u;
        x = right ? polar_g(p0, p1, lb << 31) : polar_f(p0, p1);
        if ((desc >> 17) & 1u) { // a size-16 leaf child
            float xs[16];
            gbc_allf<Q, 16>(x, base, xs);
            const uint32_t bits = leaf16_bits(desc & 0xffu, xs);
            if (w.sub == 0)
                w.put(o, 16, bits);
            return;
        }
    } else {
        x = w.psrc(4).at(i);
    }
    const bool rone = code == OP_Q16R || ((code == OP_Q16F || code == OP_Q16G) && ((desc >> 16) & 1u));
    const float xu = gxor8<Q>(x, base, i); // element i + 8 on lanes i < 8
    const float lf = polar_f(x, xu);
    float l[8];
    gbc_allf<Q, 8>(lf, base, l);
    const uint32_t bl = leaf8_bits(desc & 0xffu, l);
    const float rg = polar_g_bit(x, xu, bl, i & 7u);
    uint32_t br;
    if (!rone) {
        float r[8];
        gbc_allf<Q, 8>(rg, base, r);
        br = leaf8_bits((desc >> 8) & 0xffu, r);
    } else { // right rate-1: the signs of r (lanes 0..7 of the group)
        br = (uint32_t)(__ballot(sgn(rg) != 0) >> base) & 0xffu;
    }
    if (w.sub == 0)
        w.put(o, 16, (bl ^ br) | (br << 8));
}

template <int Q>
PCG_DEV void q16(const Cw<Q>& w, uint32_t code, uint32_t o, uint32_t desc)
{
    if (w.sub != 0)
        return;
    q16_body<Q>(w, w.psrc(4), code, o, desc);
}

// F / G / G0 from stage s into stage s-1, or the fused right rate-1 of ROneNode (:205-219)
template <int Q, typename SRC>
PCG_DEV void inner_body(const Cw<Q>& w, const SRC& src, uint32_t code, uint32_t s, uint32_t o)
{
    const uint32_t h = 1u << (s - 1);
    if (h < 4) { // h = 1, 2: one lane, scalar
        if (w.sub != 0)
            return;
        if (code == OP_RONE) {
            uint32_t lb = w.row[o >> 5] >> (o & 31u), l = 0, r = 0;
            for (uint32_t i = 0; i < h; ++i) {
                const float g = polar_g_bit(src.at(i), src.at(i + h), lb, i);
                const uint32_t rs = fbits(g) >> 31;
                l |= (((lb >> i) & 1u) ^ rs) << i;
                r |= rs << i;
            }
            w.put(o, 2 * h, l | (r << h));
            return;
        }
        float* dst = w.alpha + h;
        const uint32_t lb = code == OP_G ? (w.row[o >> 5] >> (o & 31u)) : 0u;
        for (uint32_t i = 0; i < h; ++i) {
            const float a = src.at(i), b = src.at(i + h);
            dst[i] = code == OP_F ? polar_f(a, b) : (code == OP_G ? polar_g_bit(a, b, lb, i) : a + b);
        }
        return;
    }
    const uint32_t hq = h / 4;
    if (code == OP_RONE) {
        for (uint32_t t = 0; t * Q < hq; ++t) {
            const uint32_t c = w.sub + t * Q;
            uint32_t lb = 0, rs = 0;
            if (c < hq) {
                lb = w.nib(o + 4u * c);
                rs = q_sgn4(q_g(src.ld(c), src.ld(c + hq), lb));
            }
            w.store_nibbles(o, hq, t, lb ^ rs);
            w.store_nibbles(o + h, hq, t, rs);
        }
        return;
    }
    float4* dst = reinterpret_cast<float4*>(w.alpha + h);
    uint32_t c = w.sub;
    for (; c + Q < hq; c += 2 * Q) { // two chunks in flight
        const float4 a0 = src.ld(c), b0 = src.ld(c + hq), a1 = src.ld(c + Q), b1 = src.ld(c + Q + hq);
        if (code == OP_F) {
            dst[c] = q_f(a0, b0);
            dst[c + Q] = q_f(a1, b1);
        } else if (code == OP_G) {
            dst[c] = q_g(a0, b0, w.nib(o + 4u * c));
            dst[c + Q] = q_g(a1, b1, w.nib(o + 4u * (c + Q)));
        } else {
            dst[c] = q_add(a0, b0);
            dst[c + Q] = q_add(a1, b1);
        }
    }
    if (c < hq) {
        const float4 a0 = src.ld(c), b0 = src.ld(c + hq);
        dst[c] = code == OP_F ? q_f(a0, b0) : (code == OP_G ? q_g(a0, b0, w.nib(o + 4u * c)) : q_add(a0, b0));
    }
}

template <int Q>
PCG_DEV void inner_q(Cw<Q>& w, uint32_t code, uint32_t s, uint32_t o)
{
    if (w.virt && s == w.top && code != OP_RONE) { // the root's children: recomputed where read
        w.root = code == OP_F ? 1u : (code == OP_G ? 2u : 3u);
        return;
    }
    w.with_src(s, [&](const auto& src) { inner_body<Q>(w, src, code, s, o); });
}

// COMB (bit[o+i] ^= bit[o+h+i]) / COPY0 (bit[o+i] = bit[o+h+i])
template <int Q>
PCG_DEV void bits_q(const Cw<Q>& w, uint32_t code, uint32_t s, uint32_t o)
{
    const uint32_t h = 1u << (s - 1);
    if (h >= 32) {
        for (uint32_t k = w.sub; k < h / 32; k += Q) {
            const uint32_t rv = w.row[((o + h) >> 5) + k];
            uint32_t& lv = w.row[(o >> 5) + k];
            lv = code == OP_COMB ? (lv ^ rv) : rv;
        }
    } else if (w.sub == 0) {
        const uint32_t sh = o & 31u, msk = ((1u << h) - 1u) << sh;
        const uint32_t x = w.row[o >> 5];
        const uint32_t rr = (x >> h) & msk;
        w.row[o >> 5] = code == OP_COMB ? (x ^ rr) : ((x & ~msk) | rr);
    }
}

// One schedule op (plus the parent COMBs folded into it), then a wave barrier
template <int Q>
PCG_DEV void scq_op(Cw<Q>& w, uint32_t op, uint32_t desc)
{
    const uint32_t code = op_code(op), s = op_stage(op) & 15u, o = op_off(op);
    const uint32_t up = op_stage(op) >> 4; // parent COMB levels folded into this op
    if (op_has_desc(code)) {
        if constexpr (Q >= 16)
            q16_par<Q>(w, code, o, desc);
        else if (code == OP_Q16F || code == OP_Q16G)
            q16x<Q>(w, code, o, desc);
        else
            q16<Q>(w, code, o, desc);
    } else if (code >= OP_L_R0)
        leaf_q<Q>(w, code, s, o);
    else if (code == OP_COMB || code == OP_COPY0)
        bits_q<Q>(w, code, s, o);
    else
        inner_q<Q>(w, code, s, o);
    // the folded parent COMBs, up the right spine: child (sc, oc) -> parent (sc+1, oc - 2^sc)
    for (uint32_t l = 0, sc = s, oc = o; l < up; ++l, oc -= 1u << sc, ++sc) {
        wsync();
        bits_q<Q>(w, OP_COMB, sc + 1, oc - (1u << sc));
    }
    wsync();
}

// After the walk: non-systematic re-encode, detector syndrome, info bytes and the ok flag
// of this lane's codeword.  N, W, K, kb, crc_bits and systematic are plan constants (literal
// in a plan-specialised kernel).
template <int Q>
PCG_DEV void scq_output(const Cw<Q>& w, const KernelArgs& a, uint64_t frame, bool fok, uint32_t N, uint32_t W,
                        uint32_t K, uint32_t kb, uint32_t crc_bits, int systematic)
{
    // non-systematic: re-encode x -> u in place (ButterflyFipPacked transform)
    if (!systematic) {
        for (uint32_t q = w.sub; q < W; q += Q)
            w.row[q] = transform_word(w.row[q], N);
        wsync();
        for (uint32_t d = 1; d < W; d <<= 1) {
            for (uint32_t q = w.sub; q < W; q += Q)
                if (!(q & d))
                    w.row[q] ^= w.row[q + d];
            wsync();
        }
    }
    // detector syndrome (affine GF(2) model, plan.cpp): bit r = c0_r ^ parity(cw & row_r)
    uint32_t syn = 0;
    for (uint32_t q = w.sub; q < W; q += Q) {
        const uint32_t cwq = w.row[q];
#pragma unroll 8
        for (uint32_t rb = 0; rb < crc_bits; ++rb)
            syn ^= (__builtin_popcount(cwq & a.crc_rows[rb * W + q]) & 1u) << rb;
    }
    syn = grp_xor(syn, Q) ^ a.crc_c0;
    if (fok) {
        // info bytes: the 8 positions of byte b are one 16-byte load (info_pos is padded)
        uint8_t* out = a.info + frame * kb;
        for (uint32_t b = w.sub; b < kb; b += Q) {
            const uint4 pp = *reinterpret_cast<const uint4*>(a.info_pos + 8 * b);
            const uint32_t pos[8] = { pp.x & 0xffffu, pp.x >> 16, pp.y & 0xffffu, pp.y >> 16,
                                      pp.z & 0xffffu, pp.z >> 16, pp.w & 0xffffu, pp.w >> 16 };
            uint32_t byte = 0;
#pragma unroll
            for (uint32_t q = 0; q < 8; ++q)
                if (8 * b + q < K)
                    byte |= ((w.row[pos[q] >> 5] >> (pos[q] & 31u)) & 1u) << (7 - q);
            out[b] = (uint8_t)byte;
        }
        if (a.ok && w.sub == 0)
            a.ok[frame] = syn == 0 ? 1 : 0;
    }
    wsync();
}

// PROF (development aid, PCG_OPPROF=1): s_memtime cycles and counts per op code in
// a.prof[2 * code], a.prof[2 * code + 1], kept in LDS and flushed once per wave
template <int Q, bool V, bool PROF>
__global__ void __launch_bounds__(64, 4) scq_kernel(KernelArgs a)
{
    constexpr uint32_t G = 64 / Q;
    extern __shared__ float smem_q[];
    const uint32_t lane = threadIdx.x & 63, g = lane / Q;
    const uint32_t region = scq_region(a.N, V), W = scq_words(a.N);
    unsigned long long* lprof = reinterpret_cast<unsigned long long*>(smem_q + G * region);
    if constexpr (PROF) {
        for (uint32_t b = lane; b < 128; b += 64)
            lprof[b] = 0;
        wsync();
    }
    Cw<Q> w;
    w.alpha = smem_q + g * region;
    w.row = reinterpret_cast<uint32_t*>(w.alpha + scq_alpha(a.N, V));
    w.sub = lane & (Q - 1);
    w.virt = V ? 1u : 0u;
    w.root = 1u;
    w.N = a.N;
    w.top = a.log2N;
    const uint64_t ngroups = (a.F + G - 1) / G;
    for (uint64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint64_t frame = grp * G + g;
        const bool fok = frame < a.F;
        w.y = a.llr + (fok ? frame : a.F - 1) * a.N;
        uint64_t t0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
        uint32_t nxt = ld_const(a.ops, 0);
        for (uint32_t k = 0; k < a.nops; ++k) {
            const uint32_t op = nxt; // the next schedule word is loaded while this op runs
            nxt = ld_const(a.ops, k + 1 < a.nops ? k + 1 : k);
            uint32_t desc = 0;
            if (op_has_desc(op_code(op))) {
                desc = nxt; // the descriptor word follows
                ++k;
                nxt = ld_const(a.ops, k + 1 < a.nops ? k + 1 : k);
            }
            scq_op<Q>(w, op, desc);
            if constexpr (PROF) {
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                if (lane == 0) {
                    const uint32_t code = op_code(op), s = op_stage(op) & 15u;
                    const uint32_t slot = (code & 31u) + (s >= 8 ? 32u : 0u); // large nodes apart
                    lprof[2 * slot] += t1 - t0;
                    lprof[2 * slot + 1] += 1;
                }
                t0 = t1;
            }
        }
        scq_output<Q>(w, a, frame, fok, a.N, W, a.K, a.kb, a.crc_bits, a.systematic);
        if constexpr (PROF) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            if (lane == 0) {
                lprof[2 * 15] += t1 - t0; // output stage (slot 15: no op code)
                lprof[2 * 15 + 1] += 1;
            }
        }
    }
    if constexpr (PROF) {
        wsync();
        for (uint32_t b = lane; b < 128; b += 64)
            if (lprof[b])
                atomicAdd(&a.prof[b], lprof[b]);
    }
}

#ifdef PCG_RTC
// Plan-specialised Fast-SSC kernel (jit.cpp): the source that hiprtc compiles defines the
// plan's fused schedule as PCG_RTC_OPS and its constants (PCG_RTC_Q, _V, _N, _LOG2N, _K,
// _CRC, _SYS).  The walk is unrolled at compile time: every op's code, stage, offset and
// descriptor are literals, so the dispatch branches, the schedule loads and the per-op
// address arithmetic fold away and the compiler schedules across op boundaries.
constexpr uint32_t rtc_ops[] = { PCG_RTC_OPS };
constexpr uint32_t rtc_nops = sizeof(rtc_ops) / sizeof(rtc_ops[0]);

template <int Q, uint32_t K>
PCG_DEV void scq_walk(Cw<Q>& w)
{
    if constexpr (K < rtc_nops) {
        constexpr uint32_t op = rtc_ops[K];
        constexpr bool d = op_has_desc(op_code(op));
        constexpr uint32_t desc = d ? rtc_ops[K + 1] : 0u;
        scq_op<Q>(w, op, desc);
        scq_walk<Q, K + (d ? 2u : 1u)>(w);
    }
}

} // namespace

extern "C" __global__ void __launch_bounds__(64, 4) scq_rtc_kernel(KernelArgs a)
{
    constexpr int Q = PCG_RTC_Q;
    constexpr bool V = PCG_RTC_V != 0;
    constexpr uint32_t N = PCG_RTC_N, G = 64 / Q;
    constexpr uint32_t region = scq_region(N, V), W = scq_words(N);
    extern __shared__ float smem_q[];
    const uint32_t lane = threadIdx.x & 63, g = lane / Q;
    Cw<Q> w;
    w.alpha = smem_q + g * region;
    w.row = reinterpret_cast<uint32_t*>(w.alpha + scq_alpha(N, V));
    w.sub = lane & (Q - 1);
    w.virt = V ? 1u : 0u;
    w.root = 1u;
    w.N = N;
    w.top = PCG_RTC_LOG2N;
    const uint64_t ngroups = (a.F + G - 1) / G;
    for (uint64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint64_t frame = grp * G + g;
        const bool fok = frame < a.F;
        w.y = a.llr + (fok ? frame : a.F - 1) * N;
        scq_walk<Q, 0>(w);
        scq_output<Q>(w, a, frame, fok, N, W, PCG_RTC_K, (PCG_RTC_K + 7) / 8, PCG_RTC_CRC, PCG_RTC_SYS);
    }
}

#else // host side: layouts, occupancy, launch

template <int Q, bool V>
int scq_resident(uint32_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scq_kernel<Q, V, false>, 64, lds_bytes) != hipSuccess)
        n = 0;
    return n;
}

} // namespace

// LDS dwords per wave of the LDS-resident Fast-SSC kernel (G = 64 / Q codewords; V: the
// root's children recomputed, halving the state); 0 if a wave's state does not fit a CU
uint32_t scq_layout(uint32_t N, uint32_t Q, bool V)
{
    if (N < 8 || (Q != 8 && Q != 16 && Q != 32))
        return 0;
    const uint64_t d = (uint64_t)(64 / Q) * scq_region(N, V);
    return d * 4 > 160 * 1024 ? 0u : (uint32_t)d;
}

uint64_t scq_wave_cap(uint32_t Q, bool V, uint32_t lds_dwords)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t lds = lds_dwords * 4u;
    int res = 0;
    if (V)
        res = Q == 8 ? scq_resident<8, true>(lds) : (Q == 16 ? scq_resident<16, true>(lds) : scq_resident<32, true>(lds));
    else
        res = Q == 8 ? scq_resident<8, false>(lds)
                     : (Q == 16 ? scq_resident<16, false>(lds) : scq_resident<32, false>(lds));
    uint64_t wpc = res > 0 ? (uint64_t)res : 1;
    if (wpc > 32)
        wpc = 32;
    wpc = env_wpc("PCG_SCQ_WPC", wpc);
    if (getenv("PCG_DEBUG_OCC"))
        fprintf(stderr, "[pcg] scq<%u,%d>: lds %u B, resident %d waves/CU, using %llu\n", Q, (int)V, lds, res,
                (unsigned long long)wpc);
    return (uint64_t)cus * wpc;
}

int launch_scq(const KernelArgs& a, uint32_t Q, bool V, hipStream_t stream)
{
    const uint64_t grid = a.units;
    if (grid == 0) // no waves for a non-empty batch: an error, never a silent no-op
        return a.F ? -4 : 0;
    const size_t lds = (size_t)a.wave_lds_floats * 4u + (a.prof ? 128 * sizeof(unsigned long long) : 0);
#define PCG_SCQ_LAUNCH(QV, VV)                                                                              \
    if (a.prof)                                                                                             \
        hipLaunchKernelGGL((scq_kernel<QV, VV, true>), dim3((uint32_t)grid), dim3(64), lds, stream, a);    \
    else                                                                                                    \
        hipLaunchKernelGGL((scq_kernel<QV, VV, false>), dim3((uint32_t)grid), dim3(64), lds, stream, a);
    if (V) {
        switch (Q) {
        case 8: PCG_SCQ_LAUNCH(8, true) break;
        case 16: PCG_SCQ_LAUNCH(16, true) break;
        case 32: PCG_SCQ_LAUNCH(32, true) break;
        default: return -4;
        }
    } else {
        switch (Q) {
        case 8: PCG_SCQ_LAUNCH(8, false) break;
        case 16: PCG_SCQ_LAUNCH(16, false) break;
        case 32: PCG_SCQ_LAUNCH(32, false) break;
        default: return -4;
        }
    }
#undef PCG_SCQ_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

#endif // PCG_RTC

} // namespace pcg
