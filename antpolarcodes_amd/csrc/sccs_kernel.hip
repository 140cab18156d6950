// sccs_kernel.hip -- lane-serial batched 8-bit Fast-SSC decoding (the reference's
// FastSscFipChar, src/polarcode/decoding/fastssc_fip_char.cpp) on CDNA4 (gfx950).
//
// Lane = one codeword, 64 frames per wave, walking the FastSscFip schedule (plan.cpp
// sc_char_emit) uniformly while each lane runs the reference's per-node byte loops on its
// own LLRs.  Storage as in scl_char_kernel.hip (i8_common.hpp): 16-byte lane-column units
// (stages 0..3 share one unit), LDS below Sl, a per-wave global slab above, the root's
// children recomputed from the channel (F, G, or the saturating sum of a ZeroRNode root),
// packed sign bits per lane in LDS.  Short nodes (n <= 32) keep the reference's 32-byte
// vector semantics: padding, the saturating reduction trees, minpos over the padded vector.
#include "i8_common.hpp"
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"

#ifndef PCG_RTC
#include <stdio.h>
#include <stdlib.h>
#endif

namespace pcg {

namespace {

using namespace i8;

struct CsLayout {
    uint32_t Sl, mt;
    uint32_t bits;    // LDS dword offset of the bit rows (word w of lane l at [w * 64 + l])
    uint32_t lds;     // LDS dwords per wave
    uint64_t gdwords; // global slab dwords per wave
};

__host__ __device__ inline CsLayout cs_layout(uint32_t N, uint32_t Sl)
{
    CsLayout y;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    y.mt = top - 1;
    y.Sl = Sl < y.mt ? Sl : y.mt;
    if (y.Sl < 4)
        y.Sl = y.mt < 4 ? y.mt : 4; // the shared small-stage unit stays in LDS
    y.bits = 256u * st_units(y.Sl);
    const uint32_t W = N >= 32 ? N / 32 : 1u;
    y.lds = y.bits + 64u * W;
    y.gdwords = 256ull * (st_units(y.mt) - st_units(y.Sl));
    return y;
}

template <bool I8>
struct CLane {
    uint32_t* lds;
    uint32_t* gs;
    const void* chan;
    uint32_t N, top, lane;
    CsLayout ly;
    uint32_t root = 0;

    PCG_DEV uint32_t* row() const { return lds + ly.bits + lane; }
    PCG_DEV uint4* lds_stage(uint32_t s) const { return reinterpret_cast<uint4*>(lds) + 64u * st_base(s); }
    PCG_DEV uint4* glb_stage(uint32_t s) const
    {
        return reinterpret_cast<uint4*>(gs) + 64ull * (st_base(s) - st_units(ly.Sl));
    }
    template <typename Fn>
    PCG_DEV void with_src(uint32_t s, Fn&& f) const
    {
        if (s == top)
            f(ChanSrc<I8>{ chan, N });
        else if (s == ly.mt)
            f(RootSrc<I8>{ ChanSrc<I8>{ chan, N }, row(), root });
        else if (s <= 3)
            f(SmallSrc{ lds_stage(0), lane, 1u << s });
        else if (s < ly.Sl)
            f(LdsSrc{ lds_stage(s), lane });
        else
            f(GlbSrc{ glb_stage(s), lane });
    }
    template <typename Fn>
    PCG_DEV void with_dst(uint32_t s, Fn&& f) const
    {
        if (s <= 3)
            f(SmallDst{ lds_stage(0), lane, 1u << s });
        else if (s < ly.Sl)
            f(LdsDst{ lds_stage(s), lane });
        else
            f(GlbDst{ glb_stage(s), lane });
    }
    PCG_DEV uint32_t bits_at(uint32_t o, uint32_t c) const
    {
        const uint32_t w = row()[(o >> 5) << 6];
        return c >= 32 ? w : (w >> (o & 31u)) & ((1u << c) - 1u);
    }
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
    PCG_DEV void fill(uint32_t o, uint32_t n, uint32_t pat)
    {
        if (n >= 32)
            for (uint32_t q = 0; q < n / 32; ++q)
                row()[((o >> 5) + q) << 6] = pat;
        else
            put(o, n, pat);
    }
};

// a flip "BitPtr[i] = -BitPtr[i]" changes the sign bit unless the byte is 0 or -128
PCG_DEV uint32_t flips_sign(int v) { return (v != 0 && v != -128) ? 1u : 0u; }

// lane-wise saturating accumulation of the n/32 32-byte vectors (RepetitionDecoder :225-241,
// DoubleRepetitionDecoder :249-263) into acc[8] (dwords)
template <typename Src>
PCG_DEV void vec_accumulate(const Src& src, uint32_t n, uint32_t (&acc)[8])
{
#pragma unroll
    for (int k = 0; k < 8; ++k)
        acc[k] = 0u;
    for (uint32_t c = 0; c < n / 16; c += 2) {
        const uint4 a = src.ld(c), b = src.ld(c + 1);
        acc[0] = adds4(acc[0], a.x);
        acc[1] = adds4(acc[1], a.y);
        acc[2] = adds4(acc[2], a.z);
        acc[3] = adds4(acc[3], a.w);
        acc[4] = adds4(acc[4], b.x);
        acc[5] = adds4(acc[5], b.y);
        acc[6] = adds4(acc[6], b.z);
        acc[7] = adds4(acc[7], b.w);
    }
}
// reduce_adds_epi8 (avxconvenience.h:92-101) pairs (i, i+16), (i, i+8), (i, i+4): x4 = dword 0
PCG_DEV uint32_t tree_to4(const uint32_t (&v)[8])
{
    const uint32_t a0 = adds4(v[0], v[4]), a1 = adds4(v[1], v[5]), a2 = adds4(v[2], v[6]), a3 = adds4(v[3], v[7]);
    const uint32_t b0 = adds4(a0, a2), b1 = adds4(a1, a3);
    return adds4(b0, b1);
}
PCG_DEV int reduce_adds32(const uint32_t (&v)[8])
{
    const uint32_t x4 = tree_to4(v);
    const uint32_t x2 = adds4(x4, x4 >> 16);
    return sbyte(adds4(x2, x2 >> 8), 0);
}

// a short node's 32-byte vector (n <= 32) with lanes >= n replaced by `pad`
template <typename Src>
PCG_DEV void vec32(const Src& src, uint32_t n, int pad, uint32_t (&v)[8])
{
    const uint4 a = src.ld(0);
    const uint4 b = n > 16 ? src.ld(1) : make_uint4(0u, 0u, 0u, 0u);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    for (uint32_t i = n; i < 32; ++i) {
        const uint32_t d = i >> 2, sh = 8u * (i & 3u);
        v[d] = (v[d] & ~(0xffu << sh)) | (((uint32_t)pad & 0xffu) << sh);
    }
}
PCG_DEV int vbyte(const uint32_t (&v)[8], uint32_t i) { return sbyte(v[i >> 2], i & 3u); }
PCG_DEV uint32_t vsigns(const uint32_t (&v)[8]) // sign bits of the 32 bytes
{
    uint32_t s = 0;
#pragma unroll
    for (int d = 0; d < 8; ++d)
        s |= sign4(v[d]) << (4 * d);
    return s;
}
// minpos_epu8 over 32 bytes: first byte of the smallest |x| (|-128| = 128)
PCG_DEV uint32_t minpos32(const uint32_t (&v)[8])
{
    int mv = 1 << 20;
    uint32_t mi = 0;
#pragma unroll
    for (uint32_t i = 0; i < 32; ++i) {
        const int x = vbyte(v, i), a = x < 0 ? -x : x;
        if (a < mv) {
            mv = a;
            mi = i;
        }
    }
    return mi;
}

template <typename Src, bool I8>
PCG_DEV void leaf(CLane<I8>& w, uint32_t code, const Src& src, uint32_t n, uint32_t o)
{
    switch (code) {
    case OP_C_R0:
        w.fill(o, n, 0u);
        break;
    case OP_C_R1:
        if (n <= 16) {
            w.put(o, n, sign16(src.ld(0)));
        } else {
            for (uint32_t c = 0; c < n / 16; c += 2)
                w.put(o + 16u * c, 32, sign16(src.ld(c)) | (sign16(src.ld(c + 1)) << 16));
        }
        break;
    case OP_C_REP: { // n > 32
        uint32_t acc[8];
        vec_accumulate(src, n, acc);
        w.fill(o, n, reduce_adds32(acc) < 0 ? 0xffffffffu : 0u);
        break;
    }
    case OP_C_REPS: { // RepetitionPrepare pads with 0
        uint32_t v[8];
        vec32(src, n, 0, v);
        w.fill(o, n, reduce_adds32(v) < 0 ? 0xffffffffu : 0u);
        break;
    }
    case OP_C_DREP: { // half_reduce_adds_epi8: even lanes' sum at byte 0, odd lanes' at byte 1
        uint32_t acc[8];
        vec_accumulate(src, n, acc);
        const uint32_t x4 = tree_to4(acc);
        const uint32_t x2 = adds4(x4, x4 >> 16);
        const uint32_t e = sbyte(x2, 0) < 0 ? 1u : 0u, od = sbyte(x2, 1) < 0 ? 1u : 0u;
        w.fill(o, n, e ? (od ? 0xffffffffu : 0x55555555u) : (od ? 0xaaaaaaaau : 0u));
        break;
    }
    case OP_C_SPC:    // n > 32
    case OP_C_ZSPC: { // n > 32: G0 of the halves, SPC, both halves
        const bool z = code == OP_C_ZSPC;
        const uint32_t m = z ? n / 2 : n;
        uint32_t par = 0, mi = 0;
        int mv = 1 << 20;
        for (uint32_t c = 0; c < m / 16; ++c) {
            const uint4 d = z ? adds16(src.ld(c), src.ld(c + m / 16)) : src.ld(c);
            par ^= __builtin_popcount(sign16(d));
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b) {
                const int x = byte_of(d, b), a = x < 0 ? -x : x;
                if (a < mv) {
                    mv = a;
                    mi = 16u * c + b;
                }
            }
        }
        if (mv >= 127) // the per-vector minimum is taken only below the running 127
            mi = 0;
        par &= 1u;
        uint32_t fl = 0;
        if (par) {
            const uint4 d = z ? adds16(src.ld(mi >> 4), src.ld((mi >> 4) + m / 16)) : src.ld(mi >> 4);
            fl = flips_sign(byte_of(d, mi & 15u));
        }
        for (uint32_t c = 0; c < m / 16; c += 2) {
            uint32_t sg;
            if (z)
                sg = sign16(adds16(src.ld(c), src.ld(c + m / 16))) |
                     (sign16(adds16(src.ld(c + 1), src.ld(c + 1 + m / 16))) << 16);
            else
                sg = sign16(src.ld(c)) | (sign16(src.ld(c + 1)) << 16);
            const uint32_t base = 16u * c;
            if (mi >= base && mi < base + 32u)
                sg ^= fl << (mi - base);
            w.put(o + base, 32, sg);
            if (z)
                w.put(o + m + base, 32, sg);
        }
        break;
    }
    case OP_C_SPCS: { // SpcPrepare pads with 127; minpos over the padded vector
        uint32_t v[8];
        vec32(src, n, 127, v);
        const uint32_t par = __builtin_popcount(vsigns(v)) & 1u;
        uint32_t sg = vsigns(v);
        if (par) {
            const uint32_t mi = minpos32(v);
            sg ^= flips_sign(vbyte(v, mi)) << mi;
        }
        w.put(o, n, sg);
        break;
    }
    case OP_C_ZSPCS: { // lanes >= h padded with 127 (fastssc_fip_char.cpp:372)
        const uint32_t h = n / 2;
        uint32_t x[8], v[8];
        vec32(src, n, 0, x);
        // l_i = x_i + x_{i+h} for i < h (h <= 16: all within the 32-byte vector)
        for (uint32_t i = 0; i < 32; ++i) {
            const int l = i < h ? sat8(vbyte(x, i) + vbyte(x, i + h)) : 127;
            const uint32_t d = i >> 2, sh = 8u * (i & 3u);
            v[d] = (i & 3u) == 0 ? ((uint32_t)l & 0xffu) : (v[d] | (((uint32_t)l & 0xffu) << sh));
        }
        const uint32_t par = __builtin_popcount(vsigns(v)) & 1u;
        uint32_t sg = vsigns(v);
        if (par) {
            const uint32_t mi = minpos32(v);
            sg ^= flips_sign(vbyte(v, mi)) << mi;
        }
        w.put(o, h, sg);
        w.put(o + h, h, sg);
        break;
    }
    case OP_C_ZONES: {
        const uint32_t h = n / 2;
        uint32_t x[8];
        vec32(src, n, 0, x);
        uint32_t sg = 0;
        for (uint32_t i = 0; i < h; ++i)
            sg |= (sat8(vbyte(x, i) + vbyte(x, i + h)) < 0 ? 1u : 0u) << i;
        w.put(o, h, sg);
        w.put(o + h, h, sg);
        break;
    }
    default:
        break;
    }
}

// F / G / G0 (fip_char.h:35-131) into stage s-1, or the fused right rate-1 of ROneNode
template <bool I8>
PCG_DEV void inner(CLane<I8>& w, uint32_t code, uint32_t s, uint32_t o)
{
    const uint32_t h = 1u << (s - 1);
    if (s == w.top && code != OP_RONE) {
        w.root = code == OP_F ? 0u : (code == OP_G ? 1u : 2u);
        return;
    }
    w.with_src(s, [&](const auto& src) {
        if (code == OP_RONE) { // bits: left ^= sign(G), right = sign(G)
            if (h <= 8) {
                const uint4 d = src.ld(0);
                const uint32_t lb = w.bits_at(o, h);
                uint32_t rs = 0;
                for (uint32_t k = 0; k < h; ++k)
                    rs |= (fip_g(byte_of(d, k), byte_of(d, k + h), (lb >> k) & 1u) < 0 ? 1u : 0u) << k;
                w.put(o, h, lb ^ rs);
                w.put(o + h, h, rs);
            } else {
                const uint32_t hq = h / 16;
                for (uint32_t c = 0; c < hq; ++c) {
                    const uint32_t lb = w.bits_at(o + 16u * c, 16);
                    const uint32_t rs = sign16(g16(src.ld(c), src.ld(c + hq), lb));
                    w.put(o + 16u * c, 16, lb ^ rs);
                    w.put(o + h + 16u * c, 16, rs);
                }
            }
            return;
        }
        w.with_dst(s - 1, [&](const auto& dst) {
            if (h >= 16) {
                const uint32_t hq = h >> 4;
                uint32_t c = 0;
                for (; c + 2 <= hq; c += 2) {
                    const uint4 a0 = src.ld(c), b0 = src.ld(c + hq), a1 = src.ld(c + 1), b1 = src.ld(c + 1 + hq);
                    if (code == OP_F) {
                        dst.st(c, f16(a0, b0));
                        dst.st(c + 1, f16(a1, b1));
                    } else if (code == OP_G) {
                        const uint32_t bb = w.bits_at(o + 16u * c, 32);
                        dst.st(c, g16(a0, b0, bb & 0xffffu));
                        dst.st(c + 1, g16(a1, b1, bb >> 16));
                    } else {
                        dst.st(c, adds16(a0, b0));
                        dst.st(c + 1, adds16(a1, b1));
                    }
                }
                if (c < hq) {
                    const uint4 a = src.ld(c), b = src.ld(c + hq);
                    dst.st(c, code == OP_F ? f16(a, b)
                                           : (code == OP_G ? g16(a, b, w.bits_at(o + 16u * c, 16)) : adds16(a, b)));
                }
            } else { // h = 1..8: stage s is 2h bytes of one unit
                const uint4 d = src.ld(0);
                const uint32_t nib = code == OP_G ? w.bits_at(o, h) : 0u;
                uint32_t v[2] = { 0u, 0u };
                for (uint32_t k = 0; k < h; ++k) {
                    const int l = byte_of(d, k), r = byte_of(d, k + h);
                    const int x = code == OP_F ? fip_f(l, r) : (code == OP_G ? fip_g(l, r, (nib >> k) & 1u) : sat8(l + r));
                    v[k >> 2] |= ubyte(x, k & 3u);
                }
                dst.st(0, make_uint4(v[0], v[1], 0u, 0u));
            }
        });
    });
}

template <bool I8>
PCG_DEV void bits_op(CLane<I8>& w, uint32_t code, uint32_t s, uint32_t o)
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

// One schedule word: a leaf, a Combine / Copy of the bits, or an inner F / G / G0 / ROne.
template <bool I8>
PCG_DEV void sccs_op(CLane<I8>& w, uint32_t op)
{
    const uint32_t code = op_code(op), s = op_stage(op), o = op_off(op);
    if (code >= OP_C_R0)
        w.with_src(s, [&](const auto& src) { leaf(w, code, src, 1u << s, o); });
    else if (code == OP_COMB || code == OP_COPY0)
        bits_op(w, code, s, o);
    else
        inner(w, code, s, o);
}

// (Plan-specialised kernels keep this schedule loop: the walk unrolled at compile time like
// scq_rtc_kernel's did not finish compiling within 25 minutes for N = 1024 -- each of the 177
// ops inlines its byte loops.  What a specialised plan folds is N, the layout, K, the detector
// and systematic-ness: every stage-storage test against Sl / top and every loop bound over N.)
template <bool I8>
PCG_DEV void sccs_body(const KernelArgs& a, uint32_t Sl)
{
    extern __shared__ uint32_t smem_c[];
    CLane<I8> w;
    w.lds = smem_c;
    w.N = a.N;
    w.top = a.log2N;
    w.lane = threadIdx.x & 63;
    w.ly = cs_layout(a.N, Sl);
    w.gs = reinterpret_cast<uint32_t*>(a.scratch) + (uint64_t)blockIdx.x * w.ly.gdwords;
    const uint32_t W = a.N >= 32 ? a.N / 32 : 1u;
    const uint64_t ngroups = (a.F + 63) / 64;
    for (uint64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint64_t frame = grp * 64 + w.lane;
        const bool fok = frame < a.F;
        const uint64_t fr = fok ? frame : a.F - 1;
        if constexpr (I8)
            w.chan = a.llr8 + fr * a.N;
        else
            w.chan = a.llr + fr * a.N;
        w.root = 0;
        for (uint32_t k = 0; k < a.nops; ++k)
            sccs_op<I8>(w, ld_const(a.ops, k));
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

#ifdef PCG_RTC
template <bool I8>
PCG_DEV void sccs_rtc(const KernelArgs& a)
{
    KernelArgs b = a; // the plan's constants as literals
    b.N = PCG_RTC_N;
    b.log2N = PCG_RTC_LOG2N;
    b.K = PCG_RTC_K;
    b.kb = (PCG_RTC_K + 7u) / 8u;
    b.crc_bits = PCG_RTC_CRC;
    b.systematic = PCG_RTC_SYS;
    b.nops = PCG_RTC_NOPS;
    sccs_body<I8>(b, PCG_RTC_SL);
}
} // namespace

// the plan-specialised 8-bit Fast-SSC decoder (the plan's constants and layout as literals):
// int8 channel LLRs / float LLRs quantised in the kernel (CharContainer::insertLlr)
extern "C" __global__ void __launch_bounds__(64) sccs_rtc_kernel(KernelArgs a) { sccs_rtc<true>(a); }
extern "C" __global__ void __launch_bounds__(64) sccs_rtc_kernel_f32(KernelArgs a) { sccs_rtc<false>(a); }

#else
template <bool I8>
__global__ void __launch_bounds__(64) sccs_kernel(KernelArgs a, uint32_t Sl)
{
    sccs_body<I8>(a, Sl);
}

template <bool I8>
int resident(uint32_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sccs_kernel<I8>, 64, lds_bytes) != hipSuccess)
        n = 0;
    return n;
}

} // namespace

// LDS / scratch layout of the lane-serial 8-bit Fast-SSC kernel: stages < Sl in LDS within
// PCG_SCCS_LDS_KB (default 40 KB: at N = 1024 every stored stage fits, no global slab, 4
// waves/CU -- measured 1.16e8 cw/s at 12 KB / 13 waves, 1.26e8 at 40 KB).
int sccs_layout(uint32_t N, uint32_t* lds_dwords, uint32_t* Sl, uint64_t* scratch_dwords)
{
    if (N < 8)
        return -4;
    uint32_t budget = 40u * 1024u;
    if (const char* e = getenv("PCG_SCCS_LDS_KB"))
        budget = (uint32_t)atoi(e) * 1024u;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    uint32_t best = 0;
    for (uint32_t s = 0; s <= top - 1; ++s)
        if (cs_layout(N, s).lds * 4u <= budget)
            best = s;
    if (const char* e = getenv("PCG_SCCS_SL")) { // dev override, ignored when out of range
        const uint32_t v = (uint32_t)atoi(e);
        if (v <= top - 1)
            best = v;
    }
    const CsLayout y = cs_layout(N, best);
    if (y.lds * 4u > 160u * 1024u)
        return -4;
    *lds_dwords = y.lds;
    *Sl = y.Sl;
    *scratch_dwords = y.gdwords;
    return 0;
}

uint64_t sccs_wave_cap(uint32_t lds_dwords, bool i8)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int res = i8 ? resident<true>(lds_dwords * 4u) : resident<false>(lds_dwords * 4u);
    uint64_t wpc = res > 0 ? (uint64_t)res : 1;
    if (wpc > 16)
        wpc = 16;
    wpc = env_wpc("PCG_SCCS_WPC", wpc);
    if (getenv("PCG_DEBUG_OCC"))
        fprintf(stderr, "[pcg] sccs: lds %u B, resident %d waves/CU, using %llu\n", lds_dwords * 4u, res,
                (unsigned long long)wpc);
    return (uint64_t)cus * wpc;
}

int launch_sccs(const KernelArgs& a, hipStream_t stream)
{
    const bool i8 = a.llr8 != nullptr;
    const uint64_t grid = a.units;
    if (grid == 0) // no waves for a non-empty batch: an error, never a silent no-op
        return a.F ? -4 : 0;
    const size_t lds = (size_t)a.wave_lds_floats * 4u;
    if (i8)
        hipLaunchKernelGGL((sccs_kernel<true>), dim3((uint32_t)grid), dim3(64), lds, stream, a, a.lds_stage_limit);
    else
        hipLaunchKernelGGL((sccs_kernel<false>), dim3((uint32_t)grid), dim3(64), lds, stream, a, a.lds_stage_limit);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

#endif // PCG_RTC

} // namespace pcg
