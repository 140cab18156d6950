// scl_char_kernel.hip -- lane-serial batched 8-bit fixed-point CRC-aided SCL decoding
// (the reference's SclFipChar, src/polarcode/decoding/scl_fip_char.cpp) on CDNA4.
//
// Lane = one path of one codeword; a wave decodes G = 64 / LP codewords (LP = L
// rounded up to a power of two), lanes g*LP .. g*LP+LP-1 holding codeword g's paths.
// Every codeword shares the plan's schedule and the path count after each leaf only
// depends on the schedule, so the wave walks the schedule uniformly while each lane
// runs the reference's per-path loops serially over its own LLR bytes.
//
// Path state of lane l = g*LP + p:
//   * metric (int32; the reference's `long` metrics are exact integers bounded by
//     128 N per frame; a frame starts from 0, or from the carried metric of a reused
//     decoder instance -- see DESIGN.md Q8);
//   * LLR bytes of stages s < top-1 in 16-byte units, unit c of lane l's column at
//     [(c * 64) + l] of the stage region (LDS for s < Sl, a per-wave global slab for
//     Sl <= s < top-1), so a wave-wide unit access is one contiguous 1 KiB, addressed through a 5-bit-per-stage slot table (the lane that
//     holds this path's stage s): an F/G rewrites every path's stage s-1 in its own
//     lane, a branching leaf copies the table of the path a survivor descends from --
//     the reference's lazy DataPool copy (scl_fip_char.cpp:21-171) without moving LLRs;
//   * stage top-1 (the root's children) is never stored: its bytes are recomputed from
//     the channel (F for the left child, G with the path's own left-half bits for the
//     right child) wherever they are read;
//   * the packed codeword sign bits, one LDS word column per lane.
// Leaves follow scl_fip_char.cpp literally on the bytes: Rate-0 penalty, Rate-1 / SPC
// weakest-LLR search (findWeakLlrs' swap-selection reproduced exactly from a one-pass
// candidate set: the first `passes` positions plus the `passes` smallest (value, index)
// pairs of the rest are the only elements the selection can touch), Repetition, and the
// list pruning (simplePartialSortDescending over int metrics, where ties are the rule,
// not the exception) simulated literally in LDS with a group-parallel argmax per pass.
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"
#include "i8_common.hpp"

#ifndef PCG_RTC
#include <stdio.h>
#include <stdlib.h>
#endif

namespace pcg {

namespace {

constexpr int INT_NEG = -2147483647 - 1;

// list pruning on keys in registers instead of the group's LDS candidate array (0: the LDS version,
// whose candidate region the layout then reserves: host part and kernel must be built alike, i.e. set
// it in a dev library build, not through PCG_RTC_XOPTS alone -- sclc_body refuses a mismatch)
#ifndef PCG_SCLC_RPRUNE
#define PCG_SCLC_RPRUNE 1 // measured: scl8_char 2.93e7 -> 2.99e7 cw/s (profiles/r06k_scl8_char_register_pruning_ab.txt)
#endif

// dev-only per-phase cycle profile (build with -DPCG_SCLC_PROF, run with PCG_OPPROF=1;
// tools/sclc_prof.py): buckets 1 F, 2 G, 4 COMB, 16 R0, 17 R1, 18 Rep, 19 SPC
// (candidates), 20 pruning, 21 survivors, 22 final extraction, 61 total, 62 groups
#ifdef PCG_SCLC_PROF
#define SC_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SC_ADD(prof, b, t0)                                                                    \
    do {                                                                                       \
        const uint64_t _t1 = __builtin_amdgcn_s_memtime();                                     \
        if ((prof) && (threadIdx.x & 63) == 0)                                                 \
            atomicAdd(&(prof)[(b)], (unsigned long long)(_t1 - (t0)));                         \
    } while (0)
#else
#define SC_T0(v) (void)0
#define SC_ADD(prof, b, t0) (void)0
#endif

using namespace i8;

struct Layout {
    uint32_t Sl;       // stages < Sl in LDS
    uint32_t mt;       // first recomputed stage (top-1); stages [Sl, mt) in global scratch
    uint32_t bits;     // LDS dword offset of the bit rows (word w of lane l at [w * 64 + l])
    uint32_t cand;     // LDS dword offset of the candidate keys (G groups x 9 LP x (metric << 8 | index))
    uint32_t lds;      // LDS dwords per wave
    uint64_t gdwords;  // global scratch dwords per wave
};

__host__ __device__ inline Layout make_layout(uint32_t N, uint32_t Sl)
{
    Layout y;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    y.mt = top - 1;
    y.Sl = Sl < y.mt ? Sl : y.mt;
    if (y.Sl < 4)
        y.Sl = y.mt < 4 ? y.mt : 4; // the shared small-stage unit stays in LDS
    y.bits = 256u * st_units(y.Sl);
    const uint32_t W = N >= 32 ? N / 32 : 1u;
    y.cand = y.bits + 64u * W;
    y.lds = y.cand + (PCG_SCLC_RPRUNE ? 0u : 576u); // (the register pruning needs no candidate region)
    y.gdwords = 256ull * (st_units(y.mt) - st_units(y.Sl));
    return y;
}

template <int LP, bool I8>
struct Wave {
    uint32_t* lds;
    uint32_t* gs;
    const void* chan; // this lane's frame: int8 or float
    uint32_t N, top, L;
    Layout ly;
    uint32_t lane, p, gb;
    uint64_t ptr = 0;   // slot of stage s at bits 5s
    int m = 0;          // path metric
    bool right = false; // root's right child active (recomputed stage top-1 = G)
    unsigned long long* prof = nullptr;

    PCG_DEV uint32_t* row() const { return lds + ly.bits + lane; } // word w at [w * 64]
    PCG_DEV uint32_t slot(uint32_t s) const { return gb | (uint32_t)((ptr >> (5u * s)) & 31u); }
    PCG_DEV void own(uint32_t s)
    {
        const uint32_t sh = 5u * s;
        ptr = (ptr & ~(31ull << sh)) | ((uint64_t)p << sh);
    }
    PCG_DEV uint4* lds_stage(uint32_t s) const { return reinterpret_cast<uint4*>(lds) + 64u * st_base(s); }
    PCG_DEV uint4* glb_stage(uint32_t s) const
    {
        return reinterpret_cast<uint4*>(gs) + 64ull * (st_base(s) - st_units(ly.Sl));
    }
    // call f(src) with the source of stage s of this path (uniform branch on s)
    template <typename Fn>
    PCG_DEV void with_src(uint32_t s, Fn&& f) const
    {
        if (s == top)
            f(ChanSrc<I8>{ chan, N });
        else if (s == ly.mt)
            f(RootSrc<I8>{ ChanSrc<I8>{ chan, N }, row(), right ? 1u : 0u });
        else if (s <= 3)
            f(SmallSrc{ lds_stage(0), slot(s), 1u << s });
        else if (s < ly.Sl)
            f(LdsSrc{ lds_stage(s), slot(s) });
        else
            f(GlbSrc{ glb_stage(s), slot(s) });
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
    // packed bits [o, o+c) of the own row, c <= 32 and inside one word
    PCG_DEV uint32_t bits_at(uint32_t o, uint32_t c) const
    {
        const uint32_t w = row()[(o >> 5) << 6];
        return c >= 32 ? w : (w >> (o & 31u)) & ((1u << c) - 1u);
    }
    PCG_DEV void put_row(uint32_t o, uint32_t c, uint32_t v)
    {
        uint32_t* r = row() + ((o >> 5) << 6);
        if (c >= 32) {
            *r = v;
        } else {
            const uint32_t sh = o & 31u, msk = ((1u << c) - 1u) << sh;
            *r = (*r & ~msk) | ((v << sh) & msk);
        }
    }
};

// F / G of the node at stage s (n = 2^s) into stage s-1 of the own lane
template <int LP, bool I8>
PCG_DEV void op_fg(Wave<LP, I8>& w, bool g, uint32_t s, uint32_t o, bool act)
{
    const uint32_t cs = s - 1, h = 1u << cs;
    if (s == w.top) { // the root's children are recomputed, never stored
        w.right = g;
        return;
    }
    if (act) {
        w.with_src(s, [&](const auto& src) {
            w.with_dst(cs, [&](const auto& dst) {
                if (h >= 16) {
                    const uint32_t hq = h >> 4;
                    uint32_t c = 0;
                    for (; c + 2 <= hq; c += 2) { // two units in flight
                        const uint4 a0 = src.ld(c), b0 = src.ld(c + hq), a1 = src.ld(c + 1), b1 = src.ld(c + 1 + hq);
                        if (g) {
                            const uint32_t bb = w.bits_at(o + 16u * c, 32);
                            dst.st(c, g16(a0, b0, bb & 0xffffu));
                            dst.st(c + 1, g16(a1, b1, bb >> 16));
                        } else {
                            dst.st(c, f16(a0, b0));
                            dst.st(c + 1, f16(a1, b1));
                        }
                    }
                    if (c < hq) { // hq == 1
                        const uint4 a = src.ld(c), b = src.ld(c + hq);
                        dst.st(c, g ? g16(a, b, w.bits_at(o + 16u * c, 16)) : f16(a, b));
                    }
                } else { // h = 1..8: stage s is 2h bytes of one unit
                    const uint4 d = src.ld(0);
                    const uint32_t nib = g ? w.bits_at(o, h) : 0u;
                    uint32_t v[2] = { 0u, 0u };
                    for (uint32_t k = 0; k < h; ++k) {
                        const int l = byte_of(d, k), r = byte_of(d, k + h);
                        const uint32_t q = ubyte(g ? fip_g(l, r, (nib >> k) & 1u) : fip_f(l, r), k & 3u);
                        if (k < 4)
                            v[0] |= q;
                        else
                            v[1] |= q;
                    }
                    dst.st(0, make_uint4(v[0], v[1], 0u, 0u));
                }
            });
        });
    }
    w.own(cs);
}

// ---- F / G with more lanes than paths (round 6) ------------------------------------------
// While fewer than LP paths exist (every codeword until its first branching leaf: P = 1), the
// idle lanes of a codeword group share the units of the active paths' F / G: lanes p = path
// (mod pp), pp = P rounded up to a power of two, each compute a contiguous share of the path's
// output units and write them into the path's own column (its slot table and bit row are read
// through the path's lane).  Same bytes as op_fg, fewer serial units per lane.
#ifndef PCG_SCLC_SHARE
#define PCG_SCLC_SHARE 1
#endif
#ifndef PCG_SCLC_ROOTL
#define PCG_SCLC_ROOTL 1
#endif
// waves per SIMD the register allocation must allow (<= 128 VGPRs: the 16 waves per CU that the
// 10 KB LDS budget allows)
#ifndef PCG_SCLC_MINW
#define PCG_SCLC_MINW 4
#endif
template <int LP, bool I8>
PCG_DEV void op_fg_shared(Wave<LP, I8>& w, bool g, uint32_t s, uint32_t o, uint32_t P)
{
    const uint32_t cs = s - 1, hq = 1u << (cs - 4); // output units (h = 2^cs >= 32 bytes)
    uint32_t pp = 1;
    while (pp < P)
        pp <<= 1;
    uint32_t hs = LP / pp; // lanes per path, each with an even number of units
    while (hs > 1 && 2u * hs > hq)
        hs >>= 1;
    const uint32_t path = w.p & (pp - 1), i = w.p / pp, dl = w.gb | path;
    const uint64_t pptr = __shfl(w.ptr, (int)dl, 64);
    const uint32_t* prow = w.lds + w.ly.bits + dl;   // the path's bit row, word q at [q * 64]
    const uint32_t n = hq / hs, c0 = n * i;          // this lane's units [c0, c0 + n)
    const bool act = path < P && i < hs;
    if (act) {
        const uint32_t sl = w.gb | (uint32_t)((pptr >> (5u * s)) & 31u);
        auto run = [&](const auto& src, const auto& dst) {
#pragma unroll 1
            for (uint32_t c = c0; c < c0 + n; c += 2) { // (n even: hq >= 2 hs)
                const uint4 a0 = src.ld(c), b0 = src.ld(c + hq), a1 = src.ld(c + 1), b1 = src.ld(c + 1 + hq);
                if (g) {
                    const uint32_t p0 = o + 16u * c, bb = prow[(p0 >> 5) << 6] >> (p0 & 31u);
                    dst.st(c, g16(a0, b0, bb & 0xffffu));
                    dst.st(c + 1, g16(a1, b1, bb >> 16));
                } else {
                    dst.st(c, f16(a0, b0));
                    dst.st(c + 1, f16(a1, b1));
                }
            }
        };
        auto with_dst = [&](const auto& src) {
            if (cs < w.ly.Sl)
                run(src, LdsDst{ w.lds_stage(cs), dl });
            else
                run(src, GlbDst{ w.glb_stage(cs), dl });
        };
        if (s == w.ly.mt)
            with_dst(RootSrc<I8>{ ChanSrc<I8>{ w.chan, w.N }, prow, w.right ? 1u : 0u });
        else if (s < w.ly.Sl)
            with_dst(LdsSrc{ w.lds_stage(s), sl });
        else
            with_dst(GlbSrc{ w.glb_stage(s), sl });
    }
    w.own(cs);
}

// The left child of the root (stage top-1, F(y_j, y_j+N/2): the same bytes for every path) read
// by an F / G with every lane busy (the G of the root's left child, after its left subtree): the
// LP lanes of a codeword compute its units once between them -- unit u by lane u mod LP -- and each
// path reads the two units of an output from their lane (ds_bpermute), instead of every path
// recomputing all of them (two channel loads and an F per unit).
template <int LP, bool I8, int SLOTS>
PCG_DEV void op_fg_rootl_slots(Wave<LP, I8>& w, bool g, uint32_t o, uint32_t hq, bool act)
{
    // unit u of the child (2 hq = 2 SLOTS LP units) is computed by lane u mod LP as its u[u / LP]
    const RootSrc<I8> rs{ ChanSrc<I8>{ w.chan, w.N }, w.row(), 0u };
    uint4 u[2 * SLOTS];
#pragma unroll
    for (int k = 0; k < 2 * SLOTS; ++k)
        u[k] = rs.ld((uint32_t)k * LP + w.p);
    const uint32_t cs = w.ly.mt - 1;
    auto run = [&](const auto& dst) {
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) {
#pragma unroll 1 // (one output unit at a time: the kernel stays at 4 waves per SIMD)
            for (uint32_t q = 0; q < (uint32_t)LP; ++q) {
                const int sl = (int)(w.gb | q);
                const uint32_t c = (uint32_t)k * LP + q; // output unit: a = unit c, b = unit c + hq
                const uint4 a = make_uint4(__shfl(u[k].x, sl, 64), __shfl(u[k].y, sl, 64), __shfl(u[k].z, sl, 64),
                                           __shfl(u[k].w, sl, 64));
                const uint4 b = make_uint4(__shfl(u[k + SLOTS].x, sl, 64), __shfl(u[k + SLOTS].y, sl, 64),
                                           __shfl(u[k + SLOTS].z, sl, 64), __shfl(u[k + SLOTS].w, sl, 64));
                if (!act)
                    continue;
                if (g)
                    dst.st(c, g16(a, b, w.bits_at(o + 16u * c, 16)));
                else
                    dst.st(c, f16(a, b));
            }
        }
    };
    if (cs < w.ly.Sl)
        run(LdsDst{ w.lds_stage(cs), w.lane });
    else
        run(GlbDst{ w.glb_stage(cs), w.lane });
    (void)hq;
}
template <int LP, bool I8>
PCG_DEV bool op_fg_rootl(Wave<LP, I8>& w, bool g, uint32_t s, uint32_t o, bool act)
{
    if (!PCG_SCLC_ROOTL || s < 6u || s != w.ly.mt || w.right || s == w.top)
        return false;
    const uint32_t hq = 1u << (s - 5); // output units (s >= 6); the child has 2 hq units
    if (hq < (uint32_t)LP || 2u * hq > 4u * LP)
        return false;
    if (hq == (uint32_t)LP)
        op_fg_rootl_slots<LP, I8, 1>(w, g, o, hq, act);
    else
        op_fg_rootl_slots<LP, I8, 2>(w, g, o, hq, act);
    w.own(s - 1);
    return true;
}

// CombineBits (fip_char.h:165-201) on sign bits: bit[o+i] ^= bit[o+h+i]
template <int LP, bool I8>
PCG_DEV void op_comb(Wave<LP, I8>& w, uint32_t s, uint32_t o, bool act)
{
    if (!act)
        return;
    const uint32_t h = 1u << (s - 1);
    uint32_t* r = w.row();
    if (h >= 32) {
        for (uint32_t k = 0; k < h / 32; ++k)
            r[((o >> 5) + k) << 6] ^= r[(((o + h) >> 5) + k) << 6];
    } else {
        const uint32_t sh = o & 31u, msk = ((1u << h) - 1u) << sh;
        const uint32_t x = r[(o >> 5) << 6];
        r[(o >> 5) << 6] = x ^ ((x >> h) & msk);
    }
}

// findWeakLlrs(idx, T, n, KW) (arrayfuncs.h:209-231) with T = |max(llr, -127)|: the
// swap-selection's results (T[0..KW), idx[0..KW)) from one streaming pass.  Only the
// first `lim` positions (they get displaced) and the lim smallest (value, index) pairs of
// the remaining positions can be selected, so the literal selection runs on <= 2 lim
// elements with their positions.
template <int KW, int LP, bool I8>
PCG_DEV void weak_llrs(const Wave<LP, I8>& w, uint32_t s, uint32_t n, int (&T)[KW], uint32_t (&I)[KW],
                       uint32_t& par)
{
    const uint32_t lim = n - 1 < (uint32_t)KW ? n - 1 : (uint32_t)KW;
    int v0[KW], sv[KW];
    uint32_t si[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        v0[k] = 0x7fffffff;
        sv[k] = 0x7fffffff;
        si[k] = 0xffffffffu;
    }
    par = 0;
    w.with_src(s, [&](const auto& src) {
        const uint32_t nu = n >= 16 ? n >> 4 : 1u;
        for (uint32_t c = 0; c < nu; ++c) {
            const uint4 d = src.ld(c);
#pragma unroll
            for (uint32_t b = 0; b < 16; ++b) {
                const uint32_t i = 16u * c + b;
                if (i < n) {
                    const int l = byte_of(d, b);
                    par ^= l < 0 ? 1u : 0u;
                    int t = l > -127 ? l : -127;
                    t = t < 0 ? -t : t;
                    if (i < lim) {
#pragma unroll
                        for (int k = 0; k < KW; ++k)
                            if ((uint32_t)k == i)
                                v0[k] = t;
                    } else if (t < sv[KW - 1]) { // stable insertion into the sorted set
#pragma unroll
                        for (int k = KW - 1; k >= 0; --k) {
                            const bool shift = k > 0 && t < sv[k > 0 ? k - 1 : 0];
                            if (t < sv[k]) {
                                if (shift) {
                                    sv[k] = sv[k - 1];
                                    si[k] = si[k - 1];
                                } else {
                                    sv[k] = t;
                                    si[k] = i;
                                }
                            }
                        }
                    }
                }
            }
        }
    });
    // literal swap-selection on the candidate elements: e < KW: position e (value v0),
    // e >= KW: the sorted set (position = index si)
    int ev[2 * KW];
    uint32_t ep[2 * KW], ei[2 * KW];
#pragma unroll
    for (int e = 0; e < KW; ++e) {
        ev[e] = v0[e];
        ep[e] = (uint32_t)e < lim ? (uint32_t)e : 0xffffffffu;
        ei[e] = (uint32_t)e;
        ev[KW + e] = sv[e];
        ep[KW + e] = si[e];
        ei[KW + e] = si[e];
    }
#pragma unroll
    for (int i = 0; i < KW; ++i) {
        if ((uint32_t)i < lim) {
            int bv = 0x7fffffff, bw = 0;
            uint32_t bp = 0xffffffffu;
#pragma unroll
            for (int e = 0; e < 2 * KW; ++e)
                if (ep[e] != 0xffffffffu && ep[e] >= (uint32_t)i && (ev[e] < bv || (ev[e] == bv && ep[e] < bp))) {
                    bv = ev[e];
                    bp = ep[e];
                    bw = e;
                }
#pragma unroll
            for (int e = 0; e < 2 * KW; ++e)
                if (ep[e] == (uint32_t)i)
                    ep[e] = bp;
#pragma unroll
            for (int e = 0; e < 2 * KW; ++e)
                if (e == bw)
                    ep[e] = (uint32_t)i;
            T[i] = bv;
            I[i] = ei[bw];
        } else { // after lim = n-1 passes position i holds the remaining element
            T[i] = 127;
            I[i] = (uint32_t)i;
#pragma unroll
            for (int e = 0; e < 2 * KW; ++e)
                if (ep[e] == (uint32_t)i) {
                    T[i] = ev[e];
                    I[i] = ei[e];
                }
        }
    }
}

// flip masks over (I0..I3) per candidate (scl_fip_char.cpp:451-466, 640-690)
__constant__ uint8_t kFlipR1[4] = { 0x0, 0x1, 0x2, 0x3 };
__constant__ uint8_t kFlipSpcOdd[8] = { 0x1, 0x2, 0x4, 0x8, 0x7, 0xB, 0xD, 0xE };
__constant__ uint8_t kFlipSpcEven[8] = { 0x0, 0x3, 0x5, 0x9, 0x6, 0xA, 0xC, 0xF };

template <int D>
PCG_DEV void argmax_i_step(int& v, uint32_t& q)
{
    const int ov = (int)bfly<D>((uint32_t)v);
    const uint32_t oq = bfly<D>(q);
    if (ov > v || (ov == v && oq < q)) {
        v = ov;
        q = oq;
    }
}
// (max, lowest position) over the LP lanes of a group: DPP / permlane butterflies
// (mirror partners are fine for this idempotent, commutative combine)
template <int LP>
PCG_DEV void grp_argmax_i(int& v, uint32_t& q)
{
    if constexpr (LP > 1) argmax_i_step<1>(v, q);
    if constexpr (LP > 2) argmax_i_step<2>(v, q);
    if constexpr (LP > 4) argmax_i_step<4>(v, q);
    if constexpr (LP > 8) argmax_i_step<8>(v, q);
    if constexpr (LP > 16) argmax_i_step<16>(v, q);
}

enum { LK_R1 = 0, LK_REP = 1, LK_SPC = 2 };

// A branching leaf: candidates, pruning, survivors' state (RateOneDecoder :423-505,
// RepetitionDecoder :508-580, SpcDecoder :583-726)
template <int LP, bool I8>
PCG_DEV void op_branch(Wave<LP, I8>& w, uint32_t kind, uint32_t s, uint32_t o, uint32_t& P, bool frame_ok)
{
    const uint32_t n = 1u << s;
    const uint32_t k = kind == LK_R1 ? 4u : (kind == LK_REP ? 2u : 8u);
    const uint32_t lk = kind == LK_R1 ? 2u : (kind == LK_REP ? 1u : 3u);
    const bool act = w.p < P;
    SC_T0(tb0);
    // candidate keys metric << 8 | index (|metric| < 2^23 for N <= 32768, index < 256)
    // group stride 9 LP: the 64/LP groups' lanes hit distinct LDS banks in the pruning scans
    int* KV = reinterpret_cast<int*>(w.lds + w.ly.cand) + (w.gb / LP) * (9 * LP);
    (void)KV;
    int T[4] = { 0, 0, 0, 0 };
    uint32_t I[4] = { 0, 0, 0, 0 }, par = 0;
    int kvr[8] = { 0, 0, 0, 0, 0, 0, 0, 0 }; // PCG_SCLC_RPRUNE: the keys of positions p k + j in registers
    if (act) {
        int c[8];
        const int m = w.m;
        if (kind == LK_REP) {
            int z = 0, on = 0;
            w.with_src(s, [&](const auto& src) {
                if (n >= 16) { // sum min(l,0), sum max(l,0) from sum l and sum |l|
                    int sl = 0, sa = 0;
                    for (uint32_t cc = 0; cc < (n >> 4); ++cc) {
                        const uint4 d = src.ld(cc);
                        sl += bsum(d.x) + bsum(d.y) + bsum(d.z) + bsum(d.w);
                        sa += babs(d.x) + babs(d.y) + babs(d.z) + babs(d.w);
                    }
                    z = (sl - sa) / 2;
                    on = (sl + sa) / 2;
                } else {
                    const uint4 d = src.ld(0);
                    for (uint32_t b = 0; b < n; ++b) {
                        const int l = byte_of(d, b);
                        z += l < 0 ? l : 0;
                        on += l > 0 ? l : 0;
                    }
                }
            });
            c[0] = m + z;
            c[1] = m - on;
        } else if (kind == LK_R1) {
            int t2[2];
            uint32_t i2[2];
            weak_llrs<2>(w, s, n, t2, i2, par);
            T[0] = t2[0];
            T[1] = t2[1];
            I[0] = i2[0];
            I[1] = i2[1];
            c[0] = m;
            c[1] = m - T[0];
            c[2] = m - T[1];
            c[3] = m - T[0] - T[1];
        } else {
            weak_llrs<4>(w, s, n, T, I, par);
            int mm = m, wk = 0;
            if (par) // odd parity (scl_fip_char.cpp:640-653)
                mm -= T[0];
            else
                wk = T[0];
            c[0] = mm;
            c[1] = mm - wk - T[1];
            c[2] = mm - wk - T[2];
            c[3] = mm - wk - T[3];
            c[4] = mm - T[1] - T[2];
            c[5] = mm - T[1] - T[3];
            c[6] = mm - T[2] - T[3];
            c[7] = mm - wk - T[1] - T[2] - T[3];
        }
#if PCG_SCLC_RPRUNE
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
            if (j < k)
                kvr[j] = (int)(((uint32_t)c[j] << 8) | (w.p * k + j));
#else
        for (uint32_t j = 0; j < k; ++j)
            KV[w.p * k + j] = (int)(((uint32_t)c[j] << 8) | (w.p * k + j));
#endif
    }
    wsync();
    SC_ADD(w.prof, 17 + kind, tb0);
    SC_T0(tb1);
    // simplePartialSortDescending(idx, metrics, np, size) (arrayfuncs.h:161-183)
    const uint32_t size = k * P, np = size < w.L ? size : w.L;
    const uint32_t lim = size - 1 < np ? size - 1 : np;
#if PCG_SCLC_RPRUNE
    // The same passes on the keys in registers: position q = p k + j is lane p's kvr[j].  Pass i
    // takes the group's (max metric, lowest position) among positions >= i and swaps that
    // position with position i -- a register select and two shuffles instead of LDS scans and
    // a barrier per pass.
    for (uint32_t i = 0; i < lim; ++i) {
        int bv = INT_NEG;
        uint32_t bq = 0xffffffffu;
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t q = w.p * k + j;
            if (j < k && q >= i && q < size) {
                const int v = kvr[j] >> 8;
                if (bq == 0xffffffffu || v > bv) {
                    bv = v;
                    bq = q;
                }
            }
        }
        grp_argmax_i<LP>(bv, bq);
        const uint32_t ri = i & (k - 1u), rb = bq & (k - 1u), li = i >> lk, lb = bq >> lk;
        int mi = kvr[0], mb = kvr[0];
#pragma unroll
        for (uint32_t j = 1; j < 8; ++j) {
            mi = j == ri ? kvr[j] : mi;
            mb = j == rb ? kvr[j] : mb;
        }
        const int ki = __shfl(mi, (int)(w.gb | li), 64), kb = __shfl(mb, (int)(w.gb | lb), 64);
        if (bq != i) {
#pragma unroll
            for (uint32_t j = 0; j < 8; ++j) {
                if (w.p == li && j == ri)
                    kvr[j] = kb;
                if (w.p == lb && j == rb)
                    kvr[j] = ki;
            }
        }
    }
    SC_ADD(w.prof, 20, tb1);
    SC_T0(tb2);
    // survivors: survivor q < np takes the key at position q (lane q / k, register q mod k)
    const bool surv = w.p < np;
    int key = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const int x = __shfl(kvr[j], (int)(w.gb | (w.p >> lk)), 64);
        key = j == (w.p & (k - 1u)) ? x : key;
    }
    key = surv ? key : 0;
#else
    for (uint32_t i = 0; i < lim; ++i) {
        int bv = INT_NEG;
        uint32_t bq = 0xffffffffu;
        for (uint32_t q = i + w.p; q < size; q += LP) {
            const int v = KV[q] >> 8;
            if (bq == 0xffffffffu || v > bv) {
                bv = v;
                bq = q;
            }
        }
        grp_argmax_i<LP>(bv, bq);
        if (w.p == 0 && bq != i) {
            const int t = KV[i];
            KV[i] = KV[bq];
            KV[bq] = t;
        }
        wsync();
    }
    SC_ADD(w.prof, 20, tb1);
    SC_T0(tb2);
    // survivors
    const bool surv = w.p < np;
    const int key = surv ? KV[w.p] : 0;
#endif
    const uint32_t id = (uint32_t)key & 0xffu;
    const int nm = key >> 8;
    wsync();
    const uint32_t src = id >> lk, j = id & (k - 1u);
    const uint32_t sl = w.gb | src;
    const uint64_t nptr = __shfl(w.ptr, (int)sl, 64);
    const uint32_t spar = __shfl(par, (int)sl, 64);
    uint32_t sI[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        sI[q] = __shfl(I[q], (int)sl, 64);
    // codeword prefix [0, o) from the source path (read a batch, then write it)
    const uint32_t W = w.N >= 32 ? w.N / 32 : 1u;
    const uint32_t pw = (o + 31u) >> 5;
    uint32_t* rowb = w.lds + w.ly.bits;
    for (uint32_t b0 = 0; b0 < pw; b0 += 16) {
        uint32_t t[16];
#pragma unroll
        for (uint32_t q = 0; q < 16; ++q)
            t[q] = (b0 + q < pw && b0 + q < W) ? rowb[((b0 + q) << 6) + sl] : 0u;
        wsync();
        if (surv && src != w.p)
#pragma unroll
            for (uint32_t q = 0; q < 16; ++q)
                if (b0 + q < pw && b0 + q < W)
                    rowb[((b0 + q) << 6) + w.lane] = t[q];
        wsync();
    }
    if (surv) {
        w.ptr = nptr;
        w.m = nm;
        // leaf bits: hard decisions of the source path's stage-s bytes with the
        // candidate's flips (NextBit = NextLlr, then ~ at the hinted indices)
        if (kind == LK_REP) {
            const uint32_t v = j ? 0xffffffffu : 0u;
            if (n >= 32)
                for (uint32_t q = 0; q < n / 32; ++q)
                    w.row()[((o >> 5) + q) << 6] = v;
            else
                w.put_row(o, n, v);
        } else {
            const uint32_t fm = kind == LK_R1 ? kFlipR1[j] : (spar ? kFlipSpcOdd[j] : kFlipSpcEven[j]);
            w.with_src(s, [&](const auto& src) {
                const uint32_t nu = n >= 16 ? n >> 4 : 1u;
                uint32_t acc = 0;
                for (uint32_t c = 0; c < nu; ++c) {
                    uint32_t sg = sign16(src.ld(c));
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (((fm >> q) & 1u) && (sI[q] >> 4) == c)
                            sg ^= 1u << (sI[q] & 15u);
                    if (n < 32) {
                        w.put_row(o, n, sg);
                    } else if (c & 1u) {
                        w.row()[((o + 16u * c) >> 5) << 6] = acc | (sg << 16);
                    } else {
                        acc = sg;
                    }
                }
            });
        }
    }
    P = np;
    (void)frame_ok;
    SC_ADD(w.prof, 21, tb2);
}

template <int LP, bool I8>
PCG_DEV void sclc_body(const KernelArgs& a, uint32_t Sl)
{
    extern __shared__ uint32_t smem_u[];
    constexpr uint32_t G = 64 / LP;
    Wave<LP, I8> w;
    w.lds = smem_u;
    w.N = a.N;
    w.top = a.log2N;
    w.L = a.L;
    w.ly = make_layout(a.N, Sl);
    if (w.ly.lds > a.wave_lds_floats) // a kernel built unlike the host part that sized its LDS: refuse
        return;
    w.gs = reinterpret_cast<uint32_t*>(a.scratch) + (uint64_t)blockIdx.x * w.ly.gdwords;
    w.lane = threadIdx.x & 63;
    w.prof = a.prof;
    w.p = w.lane % LP;
    w.gb = w.lane - w.p;
    const uint32_t W = a.N >= 32 ? a.N / 32 : 1u;
    // frames 0 .. F-1, or fmap[0 .. *fcount) (the adaptive decoder's second stage)
    const uint64_t Fn = a.fcount ? (uint64_t)*a.fcount : a.F;
    const uint64_t ngroups = (Fn + G - 1) / G;
    for (uint64_t grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
        const uint64_t slot = grp * G + w.lane / LP;
        const bool fok = slot < Fn;
        const uint64_t fs = fok ? slot : Fn - 1;
        const uint64_t frame = a.fmap ? (uint64_t)a.fmap[fs] : fs;
        if constexpr (I8)
            w.chan = a.llr8 + frame * a.N;
        else
            w.chan = a.llr + frame * a.N;
        w.ptr = 0;
        w.m = (int)a.metric0; // 0, or the carried metric of a reused decoder (Q8)
        w.right = false;
        uint32_t P = 1;
        SC_T0(tg0);
        for (uint32_t k = 0; k < a.nops; ++k) {
            const uint32_t op = ld_const(a.ops, k);
            const uint32_t code = op_code(op), s = op_stage(op), o = op_off(op);
            const bool act = w.p < P;
            SC_T0(to0);
            switch (code) {
            case OP_F:
            case OP_G:
                // (wave-uniform choices: P and the stage are the same for every codeword)
                if (PCG_SCLC_SHARE && 2u * P <= (uint32_t)LP && s != w.top && s >= 6u)
                    op_fg_shared(w, code == OP_G, s, o, P);
                else if (!op_fg_rootl(w, code == OP_G, s, o, act))
                    op_fg(w, code == OP_G, s, o, act);
                break;
            case OP_COMB:
                op_comb(w, s, o, act);
                break;
            case OP_CS_R0: // RateZeroDecoder :387-421: penalty, bits 0, no branching
                if (act) {
                    const uint32_t n = 1u << s;
                    int pen = 0;
                    w.with_src(s, [&](const auto& src) {
                        if (n >= 16) { // sum min(l, 0) = (sum l - sum |l|) / 2
                            int sl = 0, sa = 0;
                            for (uint32_t c = 0; c < (n >> 4); ++c) {
                                const uint4 d = src.ld(c);
                                sl += bsum(d.x) + bsum(d.y) + bsum(d.z) + bsum(d.w);
                                sa += babs(d.x) + babs(d.y) + babs(d.z) + babs(d.w);
                            }
                            pen = (sl - sa) / 2;
                        } else {
                            const uint4 d = src.ld(0);
                            for (uint32_t b = 0; b < n; ++b) {
                                const int l = byte_of(d, b);
                                pen += l < 0 ? l : 0;
                            }
                        }
                    });
                    w.m += pen;
                    if (n >= 32)
                        for (uint32_t q = 0; q < n / 32; ++q)
                            w.row()[((o >> 5) + q) << 6] = 0u;
                    else
                        w.put_row(o, n, 0u);
                }
                break;
            case OP_CS_R1:
                op_branch(w, LK_R1, s, o, P, fok);
                break;
            case OP_CS_REP:
                op_branch(w, LK_REP, s, o, P, fok);
                break;
            case OP_CS_SPC:
                op_branch(w, LK_SPC, s, o, P, fok);
                break;
            default:
                break;
            }
            wsync();
            if (code <= OP_COMB || code == OP_CS_R0)
                SC_ADD(a.prof, code & 63u, to0);
#if defined(PCG_SCLC_PROF) && defined(PCG_SCLC_PROF_POS) // dev: cycles per schedule position
            if (a.prof && w.lane == 0 && k < 3840u)
                atomicAdd(&a.prof[256u + k], (unsigned long long)(__builtin_amdgcn_s_memtime() - to0));
#endif
        }
        SC_T0(tx0);
        // extractBestPath (scl_fip_char.cpp:816-856): first path in list order whose
        // information passes the detector, else path 0
        const bool act = w.p < P;
        uint32_t* r = w.row();
        if (!a.systematic && act) { // re-encode x -> u in place (ButterflyFipPacked transform)
            for (uint32_t q = 0; q < W; ++q)
                r[q << 6] = transform_word(r[q << 6], a.N);
            for (uint32_t d = 1; d < W; d <<= 1)
                for (uint32_t q = 0; q < W; ++q)
                    if (!(q & d))
                        r[q << 6] ^= r[(q + d) << 6];
        }
        uint32_t syn = a.crc_c0;
        if (act && a.crc_bits) {
            for (uint32_t rb = 0; rb < a.crc_bits; ++rb) {
                uint32_t pc = 0;
                for (uint32_t q = 0; q < W; ++q)
                    pc += __builtin_popcount(r[q << 6] & a.crc_rows[rb * W + q]);
                syn ^= (pc & 1u) << rb;
            }
        }
        const bool pass = act && syn == 0;
        const uint64_t bal = ballot(pass);
        const uint32_t gm = (uint32_t)((bal >> w.gb) & ((LP == 64 ? ~0ull : ((1ull << LP) - 1ull))));
        const uint32_t win = gm ? (uint32_t)__builtin_ctz(gm) : 0u;
        wsync();
        if (fok) {
            const uint32_t* wr = w.lds + w.ly.bits + (w.gb | win);
            for (uint32_t b = w.p; b < a.kb; b += LP) {
                uint32_t byte = 0;
                for (uint32_t q = 0; q < 8; ++q) {
                    const uint32_t idx = 8 * b + q;
                    if (idx < a.K) {
                        const uint32_t pos = a.info_pos[idx];
                        byte |= ((wr[(pos >> 5) << 6] >> (pos & 31u)) & 1u) << (7 - q);
                    }
                }
                a.info[frame * a.kb + b] = (uint8_t)byte;
            }
            if (w.p == 0 && a.ok)
                a.ok[frame] = gm ? 1 : 0;
            if (a.metrics && w.p < a.L)
                a.metrics[frame * a.L + w.p] = act ? (float)w.m : 0.0f;
        }
        wsync();
        SC_ADD(a.prof, 22, tx0);
        SC_ADD(a.prof, 61, tg0);
#ifdef PCG_SCLC_PROF
        if (a.prof && w.lane == 0)
            atomicAdd(&a.prof[62], 1ull);
#endif
    }
}

#ifdef PCG_RTC
// the plan-specialised 8-bit list decoder (rtc.cpp sclc_rtc_source): the plan's constants and
// layout as literals, the schedule loop kept
template <bool I8>
PCG_DEV void sclc_rtc(const KernelArgs& a)
{
    KernelArgs b = a;
    b.N = PCG_RTC_N;
    b.log2N = PCG_RTC_LOG2N;
    b.K = PCG_RTC_K;
    b.kb = (PCG_RTC_K + 7u) / 8u;
    b.L = PCG_RTC_L;
    b.crc_bits = PCG_RTC_CRC;
    b.systematic = PCG_RTC_SYS;
    b.nops = PCG_RTC_NOPS;
    sclc_body<PCG_RTC_LP, I8>(b, PCG_RTC_SL);
}
} // namespace

extern "C" __global__ void __launch_bounds__(64, PCG_SCLC_MINW) scl_char_rtc_kernel(KernelArgs a) { sclc_rtc<true>(a); }
extern "C" __global__ void __launch_bounds__(64, PCG_SCLC_MINW) scl_char_rtc_kernel_f32(KernelArgs a)
{
    sclc_rtc<false>(a);
}

#else
template <int LP, bool I8>
__global__ void __launch_bounds__(64, PCG_SCLC_MINW) scl_char_kernel(KernelArgs a, uint32_t Sl)
{
    sclc_body<LP, I8>(a, Sl);
}

template <int LP, bool I8>
int resident(uint32_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, scl_char_kernel<LP, I8>, 64, lds_bytes) != hipSuccess)
        n = 0;
    return n;
}

uint32_t lp_of(uint32_t L)
{
    uint32_t lp = 2;
    while (lp < L)
        lp <<= 1;
    return lp;
}

} // namespace

// LDS / scratch layout: stages < Sl in LDS, chosen so a wave's LDS stays within
// PCG_SCLC_LDS_KB (default 10 KB: the bit rows and stages < 5 at N = 1024 -- 16 waves per CU, the
// 4-waves-per-SIMD register limit; occupancy beats LDS residency here.  Measured at N = 1024,
// L = 8 once the pruning moved to registers and its 2.3 KB candidate region went away,
// profiles/r06n_scl8_char_lds_budget_sweep.txt: 12 KB (stages < 6, 13 waves / CU) 2.21e7 cw/s,
// 10 KB 3.16-3.19e7, 9 KB (stages < 4) 3.16e7; round 5's 12 KB with the candidate region: 2.99e7).
int sclc_layout(uint32_t N, uint32_t L, uint32_t* lds_dwords, uint32_t* Sl, uint64_t* scratch_dwords)
{
    if (L < 2 || L > 32 || N < 8)
        return -4;
    uint32_t budget = (PCG_SCLC_RPRUNE ? 10u : 12u) * 1024u;
    if (const char* e = getenv("PCG_SCLC_LDS_KB"))
        budget = (uint32_t)atoi(e) * 1024u;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    uint32_t best = 0;
    for (uint32_t s = 0; s <= top - 1; ++s)
        if (make_layout(N, s).lds * 4u <= budget)
            best = s;
    if (const char* e = getenv("PCG_SCLC_SL")) { // dev override, ignored when out of range
        const uint32_t v = (uint32_t)atoi(e);
        if (v <= top - 1)
            best = v;
    }
    const Layout y = make_layout(N, best);
    if (y.lds * 4u > 160u * 1024u)
        return -4;
    *lds_dwords = y.lds;
    *Sl = y.Sl;
    *scratch_dwords = y.gdwords;
    return 0;
}

uint64_t sclc_wave_cap(uint32_t L, uint32_t lds_dwords, bool i8)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t lds = lds_dwords * 4u;
    int res = 0;
    switch (lp_of(L)) {
    case 2: res = i8 ? resident<2, true>(lds) : resident<2, false>(lds); break;
    case 4: res = i8 ? resident<4, true>(lds) : resident<4, false>(lds); break;
    case 8: res = i8 ? resident<8, true>(lds) : resident<8, false>(lds); break;
    case 16: res = i8 ? resident<16, true>(lds) : resident<16, false>(lds); break;
    default: res = i8 ? resident<32, true>(lds) : resident<32, false>(lds); break;
    }
    uint64_t wpc = res > 0 ? (uint64_t)res : 1;
    if (wpc > 16)
        wpc = 16;
    wpc = env_wpc("PCG_SCLC_WPC", wpc);
    if (getenv("PCG_DEBUG_OCC"))
        fprintf(stderr, "[pcg] sclc: lds %u B, resident %d waves/CU, using %llu\n", lds, res,
                (unsigned long long)wpc);
    return (uint64_t)cus * wpc;
}

int launch_scl_char(const KernelArgs& a, hipStream_t stream)
{
    const bool i8 = a.llr8 != nullptr;
    const uint64_t grid = a.units;
    if (grid == 0) // no waves for a non-empty batch: an error, never a silent no-op
        return a.F ? -4 : 0;
    const size_t lds = (size_t)a.wave_lds_floats * 4u;
    const uint32_t Sl = a.lds_stage_limit;
#define PCG_SCLC_LAUNCH(LPV)                                                                                   \
    if (i8)                                                                                                    \
        hipLaunchKernelGGL((scl_char_kernel<LPV, true>), dim3((uint32_t)grid), dim3(64), lds, stream, a, Sl);  \
    else                                                                                                       \
        hipLaunchKernelGGL((scl_char_kernel<LPV, false>), dim3((uint32_t)grid), dim3(64), lds, stream, a, Sl);
    switch (lp_of(a.L)) {
    case 2: PCG_SCLC_LAUNCH(2) break;
    case 4: PCG_SCLC_LAUNCH(4) break;
    case 8: PCG_SCLC_LAUNCH(8) break;
    case 16: PCG_SCLC_LAUNCH(16) break;
    case 32: PCG_SCLC_LAUNCH(32) break;
    default: return -4;
    }
#undef PCG_SCLC_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

#endif // PCG_RTC

} // namespace pcg
