// sclls_kernel.hip -- lane-serial batched CRC-aided SCL polar decoding on CDNA4 (gfx950).
//
// Lane = one path of one codeword.  A wave decodes G = 64 / LP codewords at once
// (LP = list size rounded up to a power of two), lanes g*LP .. g*LP+LP-1 holding the
// paths of codeword g.  Every codeword shares the plan's schedule and the path count
// P after each leaf only depends on the schedule, so the wave walks the schedule
// uniformly and each lane runs the reference's per-path loops literally (the AVX
// decoder's own order of operations, scl_avx_float.cpp), serially over the node's
// LLRs.  Compared with the cooperative one-codeword-per-wave kernel this removes the
// per-op address arithmetic, reductions and LDS round trips that dominated there:
// elementwise F/G become float4 streams with plenty of independent loads per lane.
//
// State of path p (lane l = g*LP + p):
//   * metric m (register);
//   * LLR stage buffers alpha[s] for stages 3 <= s < top, element chunk c (4 floats)
//     of lane l at ((c * 64) + l) * 4 -- LDS for s < Sl, a per-wave global scratch
//     slab (L2/MALL resident) for s >= Sl; stages < 3 only exist inside size-8
//     subtrees, which run in registers (OP_S_ST8);
//   * a slot table ptr (5 bits per stage): alpha[s] of path p lives in lane
//     g*LP + slot_s.  An F/G at stage s rewrites every path's alpha[s-1] (all old
//     ones are dead then) in its own lane; a branching leaf copies the table row of
//     the path each survivor descends from -- the reference's lazy DataPool copy
//     (scl_avx_float.cpp:21-171) without moving any LLRs;
//   * the path's bits.  LP < PCG_LS_DBITS_LP: the packed codeword, one LDS word column
//     per lane; a survivor of a branching leaf copies the prefix decoded so far from the
//     path it descends from.  LP >= PCG_LS_DBITS_LP (N = 4096 rows would fill the LDS):
//     lazily copied like the LLRs -- D[s] (2^s bits, stages 4 .. top) holds the two
//     decoded children of the current stage-s node, left half then right half; a child
//     (leaf or Combine) writes its half in the path's own lane, copying the left half
//     over from its slot when it writes the right one, and its own slot table bptr.
//     D[top] ends as the codeword.  Survivors copy ptr and bptr only: no bits move (D
//     stages < Sb in LDS, the rest in the global slab).
// Path selection (simplePartialSortDescending, arrayfuncs.h:161-183) is a merge of
// the LP lanes' locally sorted candidate lists; exact ties (the only case where the
// reference's swap order is observable) switch the wave to a literal simulation.
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"

#ifndef PCG_RTC
#include <stdio.h>
#include <stdlib.h>

#include <string>
#endif

namespace pcg {

namespace {

constexpr uint32_t LS_MINS = 3; // lowest memory stage: size-8 nodes

// Lanes per codeword from which the bits are lazy D buffers instead of codeword rows
// (measured round 3: SCL-32 N = 4096 6.6e5 -> 8.6e5 cw/s from 4 to 8 waves/CU; SCL-8
// N = 1024 2.22e7 -> 2.01e7, its Combines and G bit reads cost more than the row copies)
#ifndef PCG_LS_DBITS_LP
#define PCG_LS_DBITS_LP 16
#endif

// Bit words through address-space qualified pointers: an LDS and a global read behind one
// wave-uniform branch must stay two instructions (ds_read / global_load), never one flat
// load (whose wait would also drain the op's in-flight slab loads).
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(1))) uint32_t gl_u32;

// ---- layout --------------------------------------------------------------------------
struct LsLayout {
    uint32_t alpha; // 64 * (2^Sl - 2^(3+vlow)) floats (stages [3+vlow, Sl))
    uint32_t d;     // 64 * 2^(Sb-5) words: D stages [4, Sb)
    uint32_t total;
};

// Stage top-1 (the root's children) is never stored: it is recomputed from the
// channel LLRs and the path's own left-half bits wherever it is read (RootSt), which
// removes the largest per-path buffers and their HBM traffic.  Memory stages are
// [3, mtop) with mtop = top-1 (or 3 when N = 8: no memory stage at all).
// With virt = 2 stage top-2 is recomputed as well (from four channel LLRs).
constexpr __host__ __device__ inline uint32_t ls_mtop(uint32_t top, uint32_t virt)
{
    const uint32_t m = top - virt;
    return m > 3u ? m : 3u;
}
constexpr __host__ __device__ inline uint32_t ls_max_virt(uint32_t top) { return top >= 9 ? 2u : (top >= 4 ? 1u : 0u); }

// Global scratch slab of one wave: alpha stages [Sl, mtop), then the tie-fallback
// candidate list (64 * 8 values + 64 * 8 ids; rarely touched, so not worth LDS).
constexpr __host__ __device__ inline uint64_t ls_gl_alpha_floats(uint32_t mt, uint32_t Sl)
{
    return Sl < mt ? 64ull * ((1ull << mt) - (1ull << Sl)) : 0ull;
}

// The lowest stages are never stored either (vlow = 1: stage 3, N >= 64; vlow = 2: stages
// 3 and 4): every reader -- size-8 subtrees, size-8 / size-16 leaves -- recomputes its
// LLRs from the parent's chunks (F for a left child, G with the left sibling's bits for a
// right one: V3St, V4St), so the F / G ops writing them vanish and the LDS stages start at
// 3 + vlow.
constexpr __host__ __device__ inline uint32_t ls_abase(uint32_t vlow) { return 8u << vlow; } // alpha[s] at 64 * (2^s - base)

// D buffers: D[s] at word ls_doff(s) of the lane's column (D[4], D[5]: one word each, D[s]
// 2^(s-5) words at 2^(s-5); the N = 8 code's D[3] is D[4]'s word).  Stages [4, Sb) in
// LDS, [Sb, top] in the global slab (Sb >= 5).
constexpr __host__ __device__ inline uint32_t ls_doff(uint32_t s) { return s <= 4u ? 0u : 1u << (s - 5u); }
constexpr __host__ __device__ inline uint32_t ls_dlds_words(uint32_t top, uint32_t Sb)
{
    if (Sb == 0) // codeword rows: N bits per lane
        return top >= 5u ? 1u << (top - 5u) : 1u;
    const uint32_t e = Sb < top + 1u ? Sb : top + 1u;
    return e <= 5u ? 1u : 1u << (e - 5u);
}
constexpr __host__ __device__ inline uint32_t ls_dgl_words(uint32_t top, uint32_t Sb)
{
    return Sb != 0 && Sb <= top ? (1u << (top - 4u)) - (1u << (Sb - 5u)) : 0u;
}
constexpr __host__ __device__ inline LsLayout ls_layout(uint32_t top, uint32_t Sl, uint32_t vlow, uint32_t Sb)
{
    LsLayout y{};
    uint32_t o = 0;
    y.alpha = o;
    o += (1u << Sl) > ls_abase(vlow) ? 64u * ((1u << Sl) - ls_abase(vlow)) : 0u;
    y.d = o;
    o += 64u * ls_dlds_words(top, Sb);
    y.total = o;
    return y;
}

// ---- per-wave context ----------------------------------------------------------------
template <int LP>
struct Ls {
    static constexpr bool DB = LP >= PCG_LS_DBITS_LP; // lazy D buffers, else codeword rows
    float* lds;
    float* gs;        // this wave's global scratch slab
    const float* y;   // this lane's codeword channel LLRs
    uint32_t N, L, top, Sl, mt; // mt: first recomputed stage (stages >= mt are never stored)
    LsLayout ly;
    uint32_t lane, p, gb; // lane, path index in the group, group base lane
    uint32_t share;       // idle lanes help with F/G while P < LP (KernelArgs::scl_fuse bit 1)
    uint32_t stage_root;  // root-child ops stage the channel in LDS (KernelArgs::scl_fuse bit 2)
    uint32_t vlow;        // stages 3 .. 2+vlow recomputed where read (KernelArgs::scl_v3)
    uint32_t ab;          // ls_abase(vlow)
    uint32_t Sb;          // D stages [4, Sb) in LDS (KernelArgs::scl_sb)
    lds_u32* dl;          // LDS D region: word w of lane l at [(w << 6) + l]
    gl_u32* dg;           // this wave's global D region (stages >= Sb)
    uint64_t ptr;         // slot of stage s at bits 5(s-3)
    uint64_t bptr;        // D slot of stage s at bits 5(max(s,4)-4)
    bool fin;             // the root's Combine left the codeword in the LDS stage region
    float m;              // path metric
#ifdef PCG_LS_PROF
    uint64_t* lprof;
    PCG_DEV void stamp(uint32_t b, uint64_t t0) const
    {
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        if (lane == 0)
            lprof[b] += t1 - t0;
    }
#define LS_T0() const uint64_t _t0 = __builtin_amdgcn_s_memtime()
#define LS_STAMP(c, b) (c).stamp((b), _t0)
#else
#define LS_T0() (void)0
#define LS_STAMP(c, b) (void)0
#endif
    PCG_DEV uint32_t src_lane(uint32_t s) const { return gb | (uint32_t)((ptr >> (5u * (s - LS_MINS))) & 31u); }
    PCG_DEV void own(uint32_t s) { // alpha[s] of this path is now in its own lane
        const uint32_t sh = 5u * (s - LS_MINS);
        ptr = (ptr & ~(31ull << sh)) | ((uint64_t)p << sh);
    }
    PCG_DEV lds_u32* row() const { return dl + lane; } // codeword rows: word w at [w*64]
    PCG_DEV lds_u32* row_of(uint32_t l) const { return dl + l; }
    PCG_DEV static uint32_t bfield(uint32_t s) { return 5u * ((s > 4u ? s : 4u) - 4u); }
    PCG_DEV uint32_t dslot(uint32_t s) const { return (uint32_t)((bptr >> bfield(s)) & 31u); }
    PCG_DEV uint32_t dlane(uint32_t s) const { return gb | dslot(s); }
    PCG_DEV void down(uint32_t s) { // D[s] of this path is now in its own lane
        const uint32_t sh = bfield(s);
        bptr = (bptr & ~(31ull << sh)) | ((uint64_t)p << sh);
    }
    // word w of D[s] in lane l / store into the own lane (wave-uniform storage choice)
    PCG_DEV uint32_t dld(uint32_t s, uint32_t w, uint32_t l) const
    {
        const uint32_t o = ls_doff(s) + w;
        if (s < Sb)
            return dl[(o << 6) + l];
        return dg[((uint64_t)(o - (1u << (Sb - 5u))) << 6) + l];
    }
    PCG_DEV void dst(uint32_t s, uint32_t w, uint32_t v) const
    {
        const uint32_t o = ls_doff(s) + w;
        if (s < Sb)
            dl[(o << 6) + lane] = v;
        else
            dg[((uint64_t)(o - (1u << (Sb - 5u))) << 6) + lane] = v;
    }
};

#ifdef PCG_LS_PROF
// dev (op profiler): global bytes the running op requests (loads / LDS DMA in [0], stores in
// [1]), counted per wave by its first active lane over the active lanes
PCG_DEV uint32_t* ls_gb_ctr()
{
    __shared__ uint32_t n[2];
    return n;
}
PCG_DEV void ls_gb(uint32_t per_lane, int wr)
{
    const uint64_t ex = __builtin_amdgcn_read_exec();
    if (__builtin_amdgcn_mbcnt_hi((uint32_t)(ex >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ex, 0u)) == 0u)
        atomicAdd(&ls_gb_ctr()[wr], per_lane * (uint32_t)__builtin_popcountll(ex));
}
#define LS_GB(n, wr) ls_gb((n), (wr))
#else
#define LS_GB(n, wr) (void)0
#endif

// The bits of D[s] of one path, read a word at a time by G ops and recomputed right
// children (wave-uniform LDS / global choice per read).
// (Codeword rows: the row of the path's lane, relative positions from the node's offset.)
struct DBits {
    const lds_u32* l; // LDS words of D[s] (stage < Sb) or the codeword rows
    const gl_u32* g;  // global words (stage >= Sb)
    uint32_t lane;
    bool glob;
    uint32_t base; // position of relative bit 0 (rows: the node's offset)
    PCG_DEV uint32_t word(uint32_t w) const
    {
        if (glob) {
            LS_GB(4, 0);
            return g[((uint64_t)w << 6) + lane];
        }
        return l[(w << 6) + lane];
    }
    // bits from relative position i (the 32 - (i & 31) bits of its word); the word holding it
    PCG_DEV uint32_t at(uint32_t i) const { return word((base + i) >> 5) >> ((base + i) & 31u); }
    PCG_DEV uint32_t wat(uint32_t i) const { return word((base + i) >> 5); }
};
template <int LP>
PCG_DEV DBits dbits(const Ls<LP>& c, uint32_t s, uint32_t lane)
{
    DBits b;
    const uint32_t o = ls_doff(s);
    b.glob = s >= c.Sb;
    b.l = c.dl + (o << 6);
    b.g = c.dg + ((uint64_t)(b.glob ? o - (1u << (c.Sb - 5u)) : 0u) << 6);
    b.lane = lane;
    b.base = 0;
    return b;
}
template <int LP>
PCG_DEV DBits rowbits(const Ls<LP>& c, uint32_t lane, uint32_t base)
{
    return DBits{ c.dl, nullptr, lane, false, base };
}
// the bits a G of the stage-s node at o reads (its left child's) for the path in lane dl
// (D: the path's D[s] slot lane bl)
template <int LP>
PCG_DEV DBits gbits(const Ls<LP>& c, uint32_t s, uint32_t o, uint32_t dl, uint32_t bl)
{
    if constexpr (Ls<LP>::DB)
        return dbits(c, s, bl);
    else
        return rowbits(c, dl, o);
}

// Stage storages.  ld(c, l): float4 chunk c of lane l's buffer; st(c, v): own lane.
struct LdsSt {
    float* b;
    uint32_t lane;
    PCG_DEV float4 ld(uint32_t c, uint32_t l) const { return *reinterpret_cast<const float4*>(b + ((c << 6) + l) * 4u); }
    PCG_DEV void st(uint32_t c, const float4& v) const { *reinterpret_cast<float4*>(b + ((c << 6) + lane) * 4u) = v; }
};
// (Measured round 3: non-temporal buffer loads / stores for the large slab stages, meant to
// keep the small ones L2-resident, cost 3-10 % at unchanged traffic -- profiles/r03b_scl8_nt_sweep.txt.)
struct GlSt {
    float* b;
    uint32_t lane;
    PCG_DEV float4 ld(uint32_t c, uint32_t l) const
    {
        LS_GB(16, 0);
        return *reinterpret_cast<const float4*>(b + ((uint64_t)((c << 6) + l)) * 4u);
    }
    PCG_DEV void st(uint32_t c, const float4& v) const
    {
        LS_GB(16, 1);
        *reinterpret_cast<float4*>(b + ((uint64_t)((c << 6) + lane)) * 4u) = v;
    }
};
// Stages >= mt are never stored.  With virt = 1 the root's children (stage top-1)
// are recomputed wherever they are read: the left child F(y_j, y_j+N/2) is path
// independent (it is only used before any branching), the right child
// G(y_j, y_j+N/2, bit_j) uses the path's own left-half codeword bits, which every
// survivor inherits unchanged.
PCG_DEV uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
PCG_DEV float4 f4_f(const float4& a, const float4& b)
{
    return make_float4(polar_f(a.x, b.x), polar_f(a.y, b.y), polar_f(a.z, b.z), polar_f(a.w, b.w));
}
// G of 4 elements with their bits at positions k0 .. k0+3 of wb (k0 + 3 < 32)
PCG_DEV float4 f4_g(const float4& a, const float4& b, uint32_t wb, uint32_t k0 = 0)
{
    return make_float4(polar_g_bit(a.x, b.x, wb, k0), polar_g_bit(a.y, b.y, wb, k0 + 1),
                       polar_g_bit(a.z, b.z, wb, k0 + 2), polar_g_bit(a.w, b.w, wb, k0 + 3));
}

// Channel loads.  (Measured round 2: non-temporal loads here -- frames kept out of L2 to
// leave it to the stage slab -- raise traffic to 330 KB/cw and cost 10 %: the channel
// re-reads do hit L2, the slab does not; profiles/r02_scl8_nt_channel.json.)
PCG_DEV float4 chan_ld(const float* y, uint32_t c)
{
    LS_GB(16, 0);
    return reinterpret_cast<const float4*>(y)[c];
}

struct ChSt { // the channel LLRs of the lane's own codeword (stage top)
    const float* y;
    PCG_DEV float4 ld(uint32_t c, uint32_t) const { return chan_ld(y, c); }
};
template <bool LEFT>
struct RootSt { // stage top-1, left or right child of the root
    const float* y;
    DBits lb;     // the path's D[top]: the left child's bits (right child only)
    uint32_t hq1; // N/8 chunks: distance of y_j+N/2
    PCG_DEV float4 ld(uint32_t c, uint32_t) const
    {
        const float4 a = chan_ld(y, c);
        const float4 b = chan_ld(y, c + hq1);
        if (LEFT)
            return f4_f(a, b);
        return f4_g(a, b, lb.at(4u * c));
    }
};
// virt = 2, 3: stages top-2 (the codeword's quarters) and top-3 (eighths, LP >= 16) are
// recomputed from 4 / 8 channel chunks, only inside their staged F/G ops (ls_fgf_rootv).
// Any recomputed stage behind one wave-uniform switch (leaves and size-8 subtrees at
// stage top or top-1: rare, so one instantiation serves all of them).
// (The left bits are read through the live context: a survivor's reload after ls_dup
// sees the source path's D[top].)
template <int LP>
struct VirtSt {
    const Ls<LP>* cp;
    uint32_t hq1;
    bool root, left; // root: a child of the root (else the channel); left: the left one
    PCG_DEV float4 ld(uint32_t c, uint32_t l) const
    {
        if (!root)
            return ChSt{ cp->y }.ld(c, l);
        if (left)
            return RootSt<true>{ cp->y, DBits{}, hq1 }.ld(c, l);
        if constexpr (Ls<LP>::DB)
            return RootSt<false>{ cp->y, dbits(*cp, cp->top, cp->dlane(cp->top)), hq1 }.ld(c, l);
        else
            return RootSt<false>{ cp->y, rowbits(*cp, cp->lane, 0u), hq1 }.ld(c, l);
    }
};
// (virt = 2 is only planned when no leaf sits at stage top-2 or above: sclls_layout.)

// prefetch depth (float4 chunks per batch) of the streaming loops for a storage
// (Measured round 4, statically: 8 for the global slab's F / G -- one round trip fewer for a
// stage-7 G -- takes the SCL-8 kernel from 252 VGPRs to 256 with 103 spilled.)
template <typename S>
struct Pre {
    static constexpr int U = 4;
};
template <bool LEFT>
struct Pre<RootSt<LEFT>> {
    static constexpr int U = 2;
};
template <int LP>
struct Pre<VirtSt<LP>> {
    static constexpr int U = 2;
};

template <int LP>
PCG_DEV LdsSt lds_st(const Ls<LP>& c, uint32_t s)
{
    return LdsSt{ c.lds + c.ly.alpha + 64u * ((1u << s) - c.ab), c.lane };
}
template <int LP>
PCG_DEV GlSt gl_st(const Ls<LP>& c, uint32_t s)
{
    return GlSt{ c.gs + 64ull * ((1ull << s) - (1ull << c.Sl)), c.lane };
}

// Stage 3 of the path, recomputed from its stage-4 chunks (v3): chunk c of the size-8 node
// at offset o is F(a_c, a_c+2) for a left child, G(a_c, a_c+2, bits o-8+4c ..) for a right
// one, a = the path's alpha[4] (slot and bit row read through the live context, so a
// survivor's reload after ls_dup sees the source path's state).
template <int LP, typename S4>
struct V3St {
    const Ls<LP>* cp;
    S4 s4;
    uint32_t o; // the size-8 node's offset
    PCG_DEV float4 ld(uint32_t ch, uint32_t) const
    {
        const uint32_t sl = cp->src_lane(4u);
        const float4 a = s4.ld(ch, sl), b = s4.ld(ch + 2u, sl);
        if ((o & 8u) == 0u)
            return f4_f(a, b);
        // the left sibling's 8 bits: D[4] bits 0..7, or the row's o-8 ..
        if constexpr (Ls<LP>::DB)
            return f4_g(a, b, cp->dld(4u, 0u, cp->dlane(4u)) >> (4u * ch));
        const uint32_t i = (o - 8u) + 4u * ch;
        return f4_g(a, b, cp->row()[(i >> 5) << 6] >> (i & 31u));
    }
};
template <int LP, typename S4>
struct Pre<V3St<LP, S4>> {
    static constexpr int U = 2;
};
// Stage 4 recomputed from the path's stage-5 chunks (vlow = 2), the same way.
template <int LP, typename S5>
struct V4St {
    const Ls<LP>* cp;
    S5 s5;
    uint32_t o; // the size-16 node's offset
    PCG_DEV float4 ld(uint32_t ch, uint32_t) const
    {
        const uint32_t sl = cp->src_lane(5u);
        const float4 a = s5.ld(ch, sl), b = s5.ld(ch + 4u, sl);
        if ((o & 16u) == 0u)
            return f4_f(a, b);
        // the left sibling's 16 bits: D[5] bits 0..15, or the row's o-16 ..
        if constexpr (Ls<LP>::DB)
            return f4_g(a, b, cp->dld(5u, 0u, cp->dlane(5u)) >> (4u * ch));
        const uint32_t i = (o - 16u) + 4u * ch;
        return f4_g(a, b, cp->row()[(i >> 5) << 6] >> (i & 31u));
    }
};
template <int LP, typename S5>
struct Pre<V4St<LP, S5>> {
    static constexpr int U = 2;
};

// Run fn with the storage of stage s for a node at offset o (wave-uniform choice).
template <int LP, typename Fn>
PCG_DEV void with_stage(const Ls<LP>& c, uint32_t s, uint32_t o, Fn&& fn)
{
    if (c.vlow >= 2u && s <= 4u) { // stage 4 recomputed from stage 5 (and stage 3 from it)
        auto go = [&](auto s5) {
            const V4St<LP, decltype(s5)> v4{ &c, s5, o & ~15u };
            if (s == 4u)
                fn(v4);
            else
                fn(V3St<LP, decltype(v4)>{ &c, v4, o });
        };
        if (5u < c.Sl)
            go(lds_st(c, 5));
        else
            go(gl_st(c, 5));
        return;
    }
    if (c.vlow >= 1u && s == 3u) {
        if (4u < c.Sl)
            fn(V3St<LP, LdsSt>{ &c, lds_st(c, 4), o });
        else
            fn(V3St<LP, GlSt>{ &c, gl_st(c, 4), o });
        return;
    }
    if (s >= c.mt)
        fn(VirtSt<LP>{ &c, c.N >> 3, s != c.top, o < (c.N >> 1) });
    else if (s >= c.Sl)
        fn(gl_st(c, s));
    else
        fn(lds_st(c, s));
}

// ---- streaming helpers ---------------------------------------------------------------
// All loads of a batch are issued before any is used, and batch b+1 is loaded while
// batch b is processed (ping-pong).  Chunk counts are powers of two: small ones are
// one guarded batch pair; large ones run whole pairs with no guards (the last
// prefetch wraps to chunk 0), so the compiler can keep counted vmcnt waits.
template <int U, typename Src>
PCG_DEV void ld_batch(const Src& src, uint32_t c0, uint32_t nq, uint32_t sl, float4 (&x)[U])
{
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (c0 + u < nq)
            x[u] = src.ld(c0 + u, sl);
}
template <int U, typename Src>
PCG_DEV void ld_full(const Src& src, uint32_t c0, uint32_t sl, float4 (&x)[U])
{
#pragma unroll
    for (int u = 0; u < U; ++u)
        x[u] = src.ld(c0 + u, sl);
}

// fn(x, c0, valid): chunks c0 .. c0+valid-1 of [0, nq) in x[0..valid).
template <int U, typename Src, typename Fn>
PCG_DEV void stream(const Src& src, uint32_t nq, uint32_t sl, Fn&& fn)
{
    float4 xa[U], xb[U];
    if (nq <= 2 * U) {
        ld_batch<U>(src, 0, nq, sl, xa);
        ld_batch<U>(src, U, nq, sl, xb);
        fn(xa, 0u, nq < (uint32_t)U ? nq : (uint32_t)U);
        if (nq > (uint32_t)U)
            fn(xb, (uint32_t)U, nq - U);
        return;
    }
    ld_full<U>(src, 0, sl, xa);
    for (uint32_t c0 = 0; c0 < nq; c0 += 2 * U) {
        ld_full<U>(src, c0 + U, sl, xb);
        fn(xa, c0, (uint32_t)U);
        ld_full<U>(src, (c0 + 2 * U) & (nq - 1), sl, xa);
        fn(xb, c0 + U, (uint32_t)U);
    }
}

// ---- F / G ---------------------------------------------------------------------------
// Lanes working on one path's F/G.  While fewer than LP paths exist (the start of every
// codeword: P = 1 until the first branching leaf), lanes p == path (mod P') with
// P' = 2^ceil(log2 P) share the path's chunks instead of idling, writing into the
// path's own column; the path's slot table and bit row are read through its lane.
struct Share {
    uint32_t dl;   // lane of the path worked on (its column receives the output)
    uint32_t h, i; // lanes per path, this lane's index among them
    bool act;
    uint32_t sl;   // lane holding the source stage of the path
    uint32_t bl;   // lane holding the path's D[s] (a G's left bits)
    bool shr;      // lanes work on other paths (wave-uniform)
};
// lane holding D[s] of the path in lane dl
template <int LP>
PCG_DEV uint32_t path_dlane(const Ls<LP>& c, uint32_t dl, uint32_t s)
{
    const uint32_t lo = shfl((uint32_t)c.bptr, (int)dl), hi = shfl((uint32_t)(c.bptr >> 32), (int)dl);
    return c.gb | (uint32_t)(((((uint64_t)hi << 32) | lo) >> Ls<LP>::bfield(s)) & 31u);
}
template <int LP>
PCG_DEV Share ls_share(const Ls<LP>& c, uint32_t P, uint32_t s, uint32_t nch)
{
    Share w;
    if (!c.share || 2 * P > LP || nch < 4) { // every lane on its own path (wave-uniform)
        w.dl = c.lane;
        w.h = 1;
        w.i = 0;
        w.act = c.p < P;
        w.sl = c.src_lane(s < c.mt ? s : LS_MINS);
        w.bl = Ls<LP>::DB ? c.dlane(s) : 0u;
        w.shr = false;
        return w;
    }
    uint32_t pp = 1;
    while (pp < P)
        pp <<= 1;
    uint32_t h = LP / pp;
    while (h > 1 && nch < 2 * h) // at least two chunks each
        h >>= 1;
    const uint32_t path = c.p & (pp - 1);
    w.dl = c.gb | path;
    w.h = h;
    w.i = c.p / pp;
    w.act = path < P && w.i < h;
    const uint32_t lo = shfl((uint32_t)c.ptr, (int)w.dl), hi = shfl((uint32_t)(c.ptr >> 32), (int)w.dl);
    const uint64_t ptr = ((uint64_t)hi << 32) | lo;
    w.sl = c.gb | (uint32_t)((ptr >> (5u * (s - LS_MINS))) & 31u); // stages >= mt: unused
    w.bl = Ls<LP>::DB ? path_dlane(c, w.dl, s) : 0u;
    w.shr = true;
    return w;
}
// the root's left-child bits of a recomputed right child (D[top], or the row) of path w.dl
template <int LP>
PCG_DEV DBits root_bits(const Ls<LP>& c, const Share& w)
{
    if constexpr (Ls<LP>::DB)
        return dbits(c, c.top, w.shr ? path_dlane(c, w.dl, c.top) : c.dlane(c.top));
    else
        return rowbits(c, w.dl, 0u);
}
template <typename S>
struct Off { // chunks [b, ...) of a storage
    S s;
    uint32_t b;
    PCG_DEV float4 ld(uint32_t c, uint32_t l) const { return s.ld(b + c, l); }
};
template <typename S>
struct Pre<Off<S>> {
    static constexpr int U = Pre<S>::U;
};

// alpha[s-1] of every active path from alpha[s] of its slot (avx_float.h:101-164),
// h = 2^(s-1) >= 8 elements = hq float4 chunks (a power of two >= 2); the two halves
// are streamed together, chunks [cb, cb+n) by this lane.
template <int OPC, int LP, typename Src, typename Dst>
PCG_DEV void ls_fg(Src src, Dst dst, const DBits& lb, uint32_t s, const Share& w)
{
    constexpr int U = Pre<Src>::U;
    const uint32_t hq = 1u << (s - 3), n = hq / w.h, cb = n * w.i;
    const uint32_t sl = w.sl;
    if (!w.act)
        return;
    const Off<Src> sa{ src, cb }, sb{ src, hq + cb };
    auto body = [&](const float4 (&xa)[U], const float4 (&xb)[U], uint32_t c0, uint32_t valid) {
        uint32_t wb = 0;
        if (OPC == OP_G) // the batch's 4U <= 16 elements share a bit word
            wb = lb.at(4u * (cb + c0));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if ((uint32_t)u < valid) {
                const float4 r = OPC == OP_F ? f4_f(xa[u], xb[u]) : f4_g(xa[u], xb[u], wb, 4 * u);
                dst.st(cb + c0 + u, r);
            }
        }
    };
    float4 a0[U], b0[U], a1[U], b1[U];
    if (n <= 2 * U) {
        ld_batch<U>(sa, 0, n, sl, a0);
        ld_batch<U>(sb, 0, n, sl, b0);
        ld_batch<U>(sa, U, n, sl, a1);
        ld_batch<U>(sb, U, n, sl, b1);
        body(a0, b0, 0u, n < (uint32_t)U ? n : (uint32_t)U);
        if (n > (uint32_t)U)
            body(a1, b1, (uint32_t)U, n - U);
        return;
    }
    ld_full<U>(sa, 0, sl, a0);
    ld_full<U>(sb, 0, sl, b0);
    for (uint32_t c0 = 0; c0 < n; c0 += 2 * U) {
        ld_full<U>(sa, c0 + U, sl, a1);
        ld_full<U>(sb, c0 + U, sl, b1);
        body(a0, b0, c0, (uint32_t)U);
        const uint32_t nx = (c0 + 2 * U) & (n - 1);
        ld_full<U>(sa, nx, sl, a0);
        ld_full<U>(sb, nx, sl, b0);
        body(a1, b1, c0 + U, (uint32_t)U);
    }
}

template <int OPC, bool FU, int LP>
PCG_DEV void ls_rootv_op(const Ls<LP>& c, GlSt d1, GlSt d2, const DBits& lb, uint32_t s, uint32_t o, const Share& w,
                         uint32_t m);
// Recomputed quarters / eighths of a codeword with P < LP paths: the idle lanes share the
// path's staged rounds (at most as many lanes per path as a round has output chunks)
#ifndef PCG_DEEP_SHARE
#define PCG_DEEP_SHARE 1
#endif
template <int LP>
PCG_DEV uint32_t ls_root_round(const Ls<LP>& c, uint32_t s, uint32_t h, bool fused);

template <int OPC, int LP>
PCG_DEV void ls_fg_op(Ls<LP>& c, uint32_t s, uint32_t o, uint32_t P)
{
    const uint32_t d = s - 1;
    if (d >= c.mt || d < 3u + c.vlow) // recomputed where it is read
        return;
    const bool deep = s >= c.mt && s + 2u <= c.top; // a recomputed quarter / eighth
    // (those: at most as many lanes per path as one staging round has output chunks)
    const Share w = ls_share(c, P, s, deep ? PCG_DEEP_SHARE * 2u * ls_root_round(c, s, 1u, false) : 1u << (s - 3));
    const DBits lb = gbits(c, s, o, w.dl, w.bl);
    if (deep) { // its child is a leaf: staged, unfused (alpha[s-1] is global)
        const uint32_t rm = ls_root_round(c, s, w.h, false);
        if (rm) { // (always: sclls_layout plans virt >= 2 only when it stages)
            GlSt d1 = gl_st(c, d);
            d1.lane = w.dl;
            ls_rootv_op<OPC, false, LP>(c, d1, d1, lb, s, o, w, rm);
        }
        c.own(d);
        return;
    }
    auto run = [&](auto dst) {
        dst.lane = w.dl;
        if (s == c.top)
            ls_fg<OPC, LP>(ChSt{ c.y }, dst, lb, s, w);
        else if (s >= c.mt && o < (c.N >> 1))
            ls_fg<OPC, LP>(RootSt<true>{ c.y, DBits{}, c.N >> 3 }, dst, lb, s, w);
        else if (s >= c.mt)
            ls_fg<OPC, LP>(RootSt<false>{ c.y, root_bits(c, w), c.N >> 3 }, dst, lb, s, w);
        else if (s >= c.Sl)
            ls_fg<OPC, LP>(gl_st(c, s), dst, lb, s, w);
        else
            ls_fg<OPC, LP>(lds_st(c, s), dst, lb, s, w);
    };
    if (d >= c.Sl)
        run(gl_st(c, d));
    else
        run(lds_st(c, d));
    c.own(d);
}

// X (F or G) at stage s immediately followed by the child's F at stage s-1, with
// alpha[s-1] in the global slab: alpha[s-1] is stored (the child's G still needs it)
// and consumed from registers, so the F's re-read of it -- a quarter of the slab
// traffic -- disappears.  Chunk c of alpha[s-2] needs alpha[s-1] chunks c and c+hq2,
// i.e. alpha[s] chunks c, c+hq, c+hq2, c+hq2+hq.  s >= 5, so hq2 >= 2.
#ifndef PCG_FGF_U
#define PCG_FGF_U 1 // batch depth of the fused op (VGPR pressure: 2 spills 31 more registers)
#endif
template <int OPC, int LP, typename Src, typename Dst1, typename Dst2>
PCG_DEV void ls_fgf(Src src, Dst1 d1, Dst2 d2, const DBits& lb, uint32_t s, const Share& w)
{
    constexpr int U = Pre<Src>::U >= 4 ? PCG_FGF_U : 1; // four source chunks per output chunk
    const uint32_t hq = 1u << (s - 3), hq2 = hq >> 1, n = hq2 / w.h, cb = n * w.i;
    const uint32_t sl = w.sl;
    if (!w.act)
        return;
    auto load = [&](uint32_t c0, float4 (&x)[4][U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[0][u] = src.ld(cb + c0 + u, sl);
            x[1][u] = src.ld(cb + c0 + hq + u, sl);
            x[2][u] = src.ld(cb + c0 + hq2 + u, sl);
            x[3][u] = src.ld(cb + c0 + hq2 + hq + u, sl);
        }
    };
    auto body = [&](const float4 (&x)[4][U], uint32_t c0) {
        uint32_t wa = 0, wb = 0;
        if (OPC == OP_G) { // 4U <= 8 elements from an 8-aligned start share a bit word
            const uint32_t ia = 4u * (cb + c0), ib = ia + 4u * hq2;
            wa = lb.at(ia);
            wb = lb.at(ib);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float4 y0 = OPC == OP_F ? f4_f(x[0][u], x[1][u]) : f4_g(x[0][u], x[1][u], wa, 4 * u);
            const float4 y1 = OPC == OP_F ? f4_f(x[2][u], x[3][u]) : f4_g(x[2][u], x[3][u], wb, 4 * u);
            d1.st(cb + c0 + u, y0);
            d1.st(cb + c0 + hq2 + u, y1);
            d2.st(cb + c0 + u, f4_f(y0, y1));
        }
    };
    float4 xa[4][U], xb[4][U];
    load(0, xa);
    if (n <= (uint32_t)U) {
        body(xa, 0u);
        return;
    }
    for (uint32_t c0 = 0; c0 < n; c0 += 2 * U) {
        load(c0 + U, xb);
        body(xa, c0);
        load((c0 + 2 * U) & (n - 1), xa);
        body(xb, c0 + U);
    }
}

// Fused root-child op (s = top-1: alpha[s] recomputed from the channel) with the channel
// staged in LDS by global_load_lds.  Whenever a root child's F/G runs, the lower LDS
// stages are dead (nothing has started yet, or the child's left subtree is finished), so
// their region holds the channel chunks of m output chunks for every codeword of the
// wave: one DMA instruction per 1 KB and one wait per round, instead of one dependent
// register round trip per output chunk (these ops were ~22 % of SCL-8's cycles).
// Staged image: codeword g, output chunk u, source k at chunk stg_idx(8u + k, g); k < 4 are
// the channel chunks a_k (alpha[s] chunks c2, c2+hq, c2+hq2, c2+hq2+hq), k >= 4 the
// chunks a_k + N/8 (their partners y_j+N/2).
//
// Codeword-minor order (PCG_STG_GM, default): chunk i of codeword g at i*G + g, so the
// wave's read of one staged chunk -- every lane of a codeword the same address, the G
// codewords adjacent 16-byte chunks -- touches G*16 contiguous bytes: no LDS bank conflict.
// Codeword-major (i + g*per) puts the G addresses per*16 = a multiple of 128 B apart, i.e.
// on the same banks.  The DMA side is free to use either order: each lane computes its own
// source address for the LDS slot it fills.
#ifndef PCG_STG_GM
#define PCG_STG_GM 1
#endif
template <int LP>
PCG_DEV uint32_t stg_idx(uint32_t i, uint32_t g, uint32_t per)
{
#if PCG_STG_GM
    (void)per;
    return i * (64u / LP) + g;
#else
    return g * per + i;
#endif
}
// the (codeword, chunk) a staging slot f receives
template <int LP>
PCG_DEV void stg_slot(uint32_t f, uint32_t per, uint32_t& g, uint32_t& i)
{
#if PCG_STG_GM
    g = f % (64u / LP);
    i = f / (64u / LP);
#else
    g = f / per;
    i = f % per;
#endif
}
template <int OPC, bool LEFT, int LP, typename Dst2>
PCG_DEV void ls_fgf_root(const Ls<LP>& c, GlSt d1, Dst2 d2, const DBits& lb, const DBits& rb, uint32_t s,
                         const Share& w, uint32_t m)
{
    const uint32_t hq = 1u << (s - 3), hq2 = hq >> 1, hq1 = c.N >> 3;
    float* stg = c.lds + c.ly.alpha;
    const uint32_t per = 8u * m;                // chunks per codeword per round
    const uint32_t ninst = (64u / LP) * per / 64u; // DMA instructions per round
    const uint32_t n = m / w.h;                 // output chunks per lane per round
    const uint64_t yp = (uint64_t)(uintptr_t)c.y;
    const float4* stg4 = reinterpret_cast<const float4*>(stg);
    const uint32_t mg = c.lane / LP;
    // s >= 7: the bits of 8 aligned output chunks are one word per source (the root's left
    // half for a right child, the op's own G bits), loaded per 8 chunks -- the first ones
    // while the DMA runs
    const bool grp = hq2 >= 8u;
    uint32_t rw[4] = { 0, 0, 0, 0 }, lw[2] = { 0, 0 };
    auto words = [&](uint32_t cg) {
        if (!LEFT) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                rw[k] = rb.wat(4u * (cg + ((k & 1) ? hq : 0u) + ((k & 2) ? hq2 : 0u)));
        }
        if (OPC == OP_G) { // (a row's node offset is a multiple of 32 here)
            lw[0] = lb.wat(4u * cg);
            lw[1] = lb.wat(4u * (cg + hq2));
        }
    };
    for (uint32_t r = 0; r < hq2; r += m) {
        __builtin_amdgcn_s_waitcnt(0); // the previous round's LDS reads have completed
        __builtin_amdgcn_wave_barrier();
        for (uint32_t t = 0; t < ninst; ++t) {
            const uint32_t f = t * 64u + c.lane;
            uint32_t g, rem;
            stg_slot<LP>(f, per, g, rem);
            const uint32_t u = rem >> 3, k = rem & 7u;
            uint32_t a = r + u + ((k & 1u) ? hq : 0u) + ((k & 2u) ? hq2 : 0u);
            if (k & 4u)
                a += hq1;
            const uint32_t lo = shfl((uint32_t)yp, (int)(g * LP)), hi = shfl((uint32_t)(yp >> 32), (int)(g * LP));
            const float* src = reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo)) + 4u * a;
            LS_GB(16, 0);
            __builtin_amdgcn_global_load_lds(src, stg + t * 256u, 16, 0, 0);
        }
        if (grp && w.act)
            words(r + w.i * n);
        __builtin_amdgcn_s_waitcnt(0);
        __builtin_amdgcn_wave_barrier();
        if (!w.act)
            continue;
        for (uint32_t uu = 0; uu < n; ++uu) {
            const uint32_t u = w.i * n + uu, c2 = r + u;
            if (grp && uu > 0 && (uu & 7u) == 0)
                words(c2);
            const uint32_t gs = 4u * (c2 & 7u);
            float4 yv[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                yv[k] = stg4[stg_idx<LP>(u * 8u + k, mg, per)];
            float4 x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (LEFT) {
                    x[k] = f4_f(yv[k], yv[k + 4]);
                } else {
                    const uint32_t a = c2 + ((k & 1) ? hq : 0u) + ((k & 2) ? hq2 : 0u);
                    x[k] = (grp ? f4_g(yv[k], yv[k + 4], rw[k], gs) : f4_g(yv[k], yv[k + 4], rb.at(4u * a)));
                }
            }
            uint32_t wa = 0, wb = 0;
            if (OPC == OP_G) {
                const uint32_t ia = 4u * c2, ib = ia + 4u * hq2;
                wa = grp ? lw[0] : lb.at(ia); // (grp: bit gs + j of the word, else bit j)
                wb = grp ? lw[1] : lb.at(ib);
            }
            // x[1] = alpha[s] chunk c2+hq pairs with x[0]; x[2], x[3] = chunks c2+hq2, c2+hq2+hq
            const float4 y0 = OPC == OP_F ? f4_f(x[0], x[1]) : f4_g(x[0], x[1], wa, grp ? gs : 0u);
            const float4 y1 = OPC == OP_F ? f4_f(x[2], x[3]) : f4_g(x[2], x[3], wb, grp ? gs : 0u);
            d1.st(c2, y0);
            d1.st(c2 + hq2, y1);
            d2.st(c2, f4_f(y0, y1));
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
}

// Output chunks per staging round of ls_fgf_root, or 0 when it does not apply: the
// LDS stages' region must hold a round, hold no output, and give every lane a chunk.
template <int LP>
PCG_DEV uint32_t ls_root_round(const Ls<LP>& c, uint32_t s, uint32_t h, bool fused)
{
    // (unfused: only a recomputed quarter's / eighth's X, whose output alpha[s-1] must not
    // be in the region)
    if (!c.stage_root || s != c.mt || s == c.top || s - (fused ? 2u : 1u) < c.Sl || (1u << c.Sl) <= c.ab)
        return 0;
    const uint32_t region = 4u * 64u * ((1u << c.Sl) - c.ab); // bytes
    const uint32_t V = c.top - s;                                 // 1: a root child
    const uint32_t k = V == 1 ? 8u : (fused ? 4u : 2u) << V;      // channel chunks per output chunk
    uint32_t m = fused ? 1u << (s - 4) : 1u << (s - 3);          // output chunks of the op
    while (m > 1 && (64u / LP) * k * m * 16u > region)
        m >>= 1;
    const uint32_t need = h > LP / k ? h : LP / k;
    return (64u / LP) * k * m * 16u <= region && m >= need && m >= 1 ? m : 0u;
}

// virt >= 2: an F/G on a node of stage s = top-V (V = 2: a quarter of the codeword, 3: an
// eighth), staged like ls_fgf_root.  Alpha[s] chunk a_k (k < KS: c2, c2+hq, and, fused with
// the child's F, c2+hq2, c2+hq2+hq) is rebuilt from the 2^V channel chunks a_k + off(j),
// off(j) = sum over the set bits l-1 of j of h_l = N/2^(l+2) chunks, staged at index
// (u*KS + k)*2^V + j.  Level l = 1..V combines pairs along h_l: F, or G (RM bit l-1) with
// the bits of the left child of the level-l ancestor -- vb[l-1]: the root's left half, then
// D[top-1] / the row at that node, D[top-2] / ...  FU = false: the X alone (its child is a
// leaf): output chunk c2 < hq of alpha[s-1] from alpha[s] chunks c2, c2+hq.
// Double-buffered rounds (PCG_STG_DB): the staging region is split in two halves of m/2 output
// chunks each; round k+1's DMA is issued into one half before round k computes from the other,
// and the wave waits for all but that round's DMA instructions (s_waitcnt vmcnt(ninst)) -- so a
// round's fetch latency overlaps the previous round's arithmetic instead of adding to it.
#ifndef PCG_STG_DB
#define PCG_STG_DB 1
#endif
#ifndef PCG_STG_TAIL_DRAIN
#define PCG_STG_TAIL_DRAIN 0 // 1: the recomputed-node ops end waiting for their stores too
#endif
#ifndef PCG_LS_STAGGER
#define PCG_LS_STAGGER 2 // start-stagger step (x s_sleep 127) per pseudo-random unit, 0: off (sclls_body)
#endif
#ifndef PCG_STG_RING
#define PCG_STG_RING 2 // at most this many buffers (measured: 3 buffers -1 % against 2 on config 3, r05g)
#endif
// s_waitcnt: vector memory counter <= n (loads, stores and LDS DMA, in issue order), the others
// not waited for (gfx9 encoding: vmcnt [3:0] and [15:14], expcnt [6:4], lgkmcnt [11:8])
#define PCG_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | ((((n) >> 4) & 3) << 14) | (7 << 4) | (15 << 8))
// One LDS-DMA instruction (16 B per lane, lane-linear 1 KiB at lds), written as inline asm: the
// compiler's own wait bookkeeping does not see it, so it does not drain it (vmcnt(0)) before
// every LDS read of the other half -- the double-buffered rounds count it themselves (wait_vm,
// then a barrier, then the reads).  M0 is set and restored in the same statement
// (cdna_hip_programming.md, LDS-DMA recipe).
PCG_DEV void glds16(const float* src, float* lds)
{
    LS_GB(16, 0);
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)lds);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(dst)
                 : "memory");
}
PCG_DEV void wait_vm(uint32_t n) // (wave-uniform n <= 63; the instruction takes an immediate)
{
    switch (n) {
    case 1: PCG_WAIT_VM(1); break;
    case 2: PCG_WAIT_VM(2); break;
    case 3: PCG_WAIT_VM(3); break;
    case 4: PCG_WAIT_VM(4); break;
    case 5: PCG_WAIT_VM(5); break;
    case 6: PCG_WAIT_VM(6); break;
    case 7: PCG_WAIT_VM(7); break;
    case 8: PCG_WAIT_VM(8); break;
    case 9: PCG_WAIT_VM(9); break;
    case 10: PCG_WAIT_VM(10); break;
    case 11: PCG_WAIT_VM(11); break;
    case 12: PCG_WAIT_VM(12); break;
    case 13: PCG_WAIT_VM(13); break;
    case 14: PCG_WAIT_VM(14); break;
    case 15: PCG_WAIT_VM(15); break;
    case 16: PCG_WAIT_VM(16); break;
    case 17: PCG_WAIT_VM(17); break;
    case 18: PCG_WAIT_VM(18); break;
    case 19: PCG_WAIT_VM(19); break;
    case 20: PCG_WAIT_VM(20); break;
    case 21: PCG_WAIT_VM(21); break;
    case 22: PCG_WAIT_VM(22); break;
    case 23: PCG_WAIT_VM(23); break;
    case 24: PCG_WAIT_VM(24); break;
    case 25: PCG_WAIT_VM(25); break;
    case 26: PCG_WAIT_VM(26); break;
    case 27: PCG_WAIT_VM(27); break;
    case 28: PCG_WAIT_VM(28); break;
    case 29: PCG_WAIT_VM(29); break;
    case 30: PCG_WAIT_VM(30); break;
    case 31: PCG_WAIT_VM(31); break;
    case 32: PCG_WAIT_VM(32); break;
    case 33: PCG_WAIT_VM(33); break;
    case 34: PCG_WAIT_VM(34); break;
    case 35: PCG_WAIT_VM(35); break;
    case 36: PCG_WAIT_VM(36); break;
    case 37: PCG_WAIT_VM(37); break;
    case 38: PCG_WAIT_VM(38); break;
    case 39: PCG_WAIT_VM(39); break;
    case 40: PCG_WAIT_VM(40); break;
    case 41: PCG_WAIT_VM(41); break;
    case 42: PCG_WAIT_VM(42); break;
    case 43: PCG_WAIT_VM(43); break;
    case 44: PCG_WAIT_VM(44); break;
    case 45: PCG_WAIT_VM(45); break;
    case 46: PCG_WAIT_VM(46); break;
    case 47: PCG_WAIT_VM(47); break;
    case 48: PCG_WAIT_VM(48); break;
    case 49: PCG_WAIT_VM(49); break;
    case 50: PCG_WAIT_VM(50); break;
    case 51: PCG_WAIT_VM(51); break;
    case 52: PCG_WAIT_VM(52); break;
    case 53: PCG_WAIT_VM(53); break;
    case 54: PCG_WAIT_VM(54); break;
    case 55: PCG_WAIT_VM(55); break;
    case 56: PCG_WAIT_VM(56); break;
    case 57: PCG_WAIT_VM(57); break;
    case 58: PCG_WAIT_VM(58); break;
    case 59: PCG_WAIT_VM(59); break;
    case 60: PCG_WAIT_VM(60); break;
    case 61: PCG_WAIT_VM(61); break;
    case 62: PCG_WAIT_VM(62); break;
    case 63: PCG_WAIT_VM(63); break;
    default: __builtin_amdgcn_s_waitcnt(0); break; // (0, or any larger count: wait for all)
    }
}

// The leading recompute levels whose combine is F (RM's low zero bits) do not depend on the path:
// they are computed once per codeword, by the whole wave right after a round lands (any lane,
// any codeword: the staged groups are spread over the 64 lanes), in place in the staged image --
// so every path reads J >> L0 chunks per source instead of J and skips those levels.  (Config 3:
// the codeword's first two quarters, whose level 1 is F(y_j, y_j+N/2); the first quarter's
// level 2 too.)
#ifndef PCG_STG_SHARED_F
#define PCG_STG_SHARED_F 1
#endif
template <int V, int RM>
constexpr uint32_t rm_lead_f()
{
    uint32_t l = 0;
    while (PCG_STG_SHARED_F && l < (uint32_t)V && !((RM >> l) & 1))
        ++l;
    return l;
}

template <int OPC, int V, int RM, bool FU, int LP>
PCG_DEV void ls_fgf_rootv(const Ls<LP>& c, GlSt d1, GlSt d2, const DBits& lb, const DBits (&vb)[3], uint32_t s,
                          const Share& w, uint32_t m)
{
    constexpr uint32_t KS = FU ? 4u : 2u, J = 1u << V;
    constexpr uint32_t L0 = rm_lead_f<V, RM>(), J0 = J >> L0; // shared levels, chunks left per source
    const uint32_t hq = 1u << (s - 3), hq2 = hq >> 1;
    const uint32_t hl[3] = { c.N >> 3, c.N >> 4, c.N >> 5 };
    const uint32_t nout = FU ? hq2 : hq;           // output chunks of the op
    float* stg = c.lds + c.ly.alpha;
    // (wave-uniform) a ring of NB buffers of m/2 output chunks each -- as many as the LDS stage
    // region holds, at most 4 -- when a buffer still gives every lane an output chunk: NB-1 rounds'
    // fetches stay in flight while one computes (the ops are bound by the fetch latency: 32 KB of
    // channel per wave and op through a 12 KB region, config 3).  With codeword rows only: with D
    // buffers (LP >= 16) the level bits are global loads that the compiler waits for with vmcnt(0),
    // which drains the in-flight rounds as well (measured with two buffers, config 5: 1.244e6 ->
    // 1.203e6 cw/s; config 3, rows: 2.844e7 -> 2.874e7; profiles/r05b_*)
    // (The double-buffered wait counts this op's global stores: every computed round issues exactly
    // n * (FU ? 3 : 1) store instructions per active lane -- d1 / d2 below, unconditional.  The dev
    // ablations that skip or replace them (PCG_DEV_ABL_DEEP 2 / 3) therefore run single-buffered,
    // with full waits, so their timings carry no fetch race.)
#if defined(PCG_DEV_ABL_DEEP) && (PCG_DEV_ABL_DEEP == 2 || PCG_DEV_ABL_DEEP == 3)
    const bool dbl = false;
#else
    const bool dbl = PCG_STG_DB && !Ls<LP>::DB && (m >> 1) >= w.h && (64u / LP) * KS * J * (m >> 1) >= 64u;
#endif
    uint32_t NB = 1;
    if (dbl) {
        m >>= 1;
        const uint32_t region = 4u * 64u * ((1u << c.Sl) - c.ab);    // bytes
        NB = region / ((64u / LP) * KS * J * m * 16u);
        NB = NB > (uint32_t)PCG_STG_RING ? (uint32_t)PCG_STG_RING : NB;
    }
    const uint32_t per = KS * J * m;               // chunks per codeword per round
    const uint32_t ninst = (64u / LP) * per / 64u; // DMA instructions per round
    const uint32_t hoff = dbl ? ninst * 256u : 0u; // floats: one buffer
    const uint32_t n = m / w.h;                    // output chunks per lane per round
    const uint64_t yp = (uint64_t)(uintptr_t)c.y;
    const float4* stg4 = reinterpret_cast<const float4*>(stg);
    const uint32_t mg = c.lane / LP;
    auto koff = [&](uint32_t k) { return ((k & 1u) ? hq : 0u) + ((k & 2u) ? hq2 : 0u); };
    // bit words of 8 aligned output chunks (s >= 7: every offset a multiple of 8 chunks):
    // level l's J >> l outputs at bw[k][J - (J >> (l-1)) + i]
    uint32_t bw[KS][J], lw[2] = { 0, 0 };
#pragma unroll
    for (uint32_t k = 0; k < KS; ++k)
#pragma unroll
        for (uint32_t i = 0; i < J; ++i)
            bw[k][i] = 0;
    auto words = [&](uint32_t cg) {
#pragma unroll
        for (uint32_t k = 0; k < KS; ++k) {
            const uint32_t a = cg + koff(k);
#pragma unroll
            for (int l = 1; l <= V; ++l) {
                if (!((RM >> (l - 1)) & 1))
                    continue;
#pragma unroll
                for (uint32_t i = 0; i < (J >> l); ++i) {
                    uint32_t off = 0;
#pragma unroll
                    for (int q = l + 1; q <= V; ++q)
                        off += ((i >> (q - l - 1)) & 1u) ? hl[q - 1] : 0u;
                    bw[k][J - (J >> (l - 1)) + i] = vb[l - 1].wat(4u * (a + off));
                }
            }
        }
        if (OPC == OP_G) {
            lw[0] = lb.wat(4u * cg);
            if (FU)
                lw[1] = lb.wat(4u * (cg + hq2));
        }
    };
    // round r's channel chunks into the half at float offset hb
    auto issue = [&](uint32_t r, uint32_t hb) {
#if defined(PCG_DEV_ABL_DEEP) && PCG_DEV_ABL_DEEP == 1 // dev ablation (wrong results): no channel DMA
        return;
#endif
        for (uint32_t t = 0; t < ninst; ++t) {
            const uint32_t f = t * 64u + c.lane;
            uint32_t g, rem;
            stg_slot<LP>(f, per, g, rem);
            const uint32_t u = rem / (KS * J), k = (rem / J) % KS, j = rem % J;
            uint32_t a = r + u + koff(k);
#pragma unroll
            for (int l = 1; l <= V; ++l)
                a += ((j >> (l - 1)) & 1u) ? hl[l - 1] : 0u;
            const uint32_t lo = shfl((uint32_t)yp, (int)(g * LP)), hi = shfl((uint32_t)(yp >> 32), (int)(g * LP));
            const float* src = reinterpret_cast<const float*>((uintptr_t)(((uint64_t)hi << 32) | lo)) + 4u * a;
            if (PCG_STG_DB && !Ls<LP>::DB) // (every round explicitly waited for: s_waitcnt / wait_vm below)
                glds16(src, stg + hb + t * 256u);
            else {
                LS_GB(16, 0);
                __builtin_amdgcn_global_load_lds(src, stg + hb + t * 256u, 16, 0, 0);
            }
        }
    };
    // round k lives in buffer k % NB; the first NB-1 rounds are fetched up front
    const uint32_t R = (nout + m - 1) / m;
    if (dbl) {
        __builtin_amdgcn_s_waitcnt(0); // (the region's previous readers have completed)
        __builtin_amdgcn_wave_barrier();
        for (uint32_t k = 0; k + 1 < NB && k < R; ++k)
            issue(k * m, k * hoff);
    }
    uint32_t hb = 0, kb = 0;
    for (uint32_t r = 0, k = 0; r < nout; r += m, ++k) {
        if (!dbl) {
            __builtin_amdgcn_s_waitcnt(0); // the previous round's LDS reads have completed
            __builtin_amdgcn_wave_barrier();
            issue(r, 0);
        }
        if (w.act)
            words(r + w.i * n);
        if (dbl) {
            // the buffer of round k-1 (its readers and writers have completed) takes round
            // k+NB-1; then wait for everything but the rounds still in flight behind round k
            const uint32_t ahead = R - 1 - k < NB - 1 ? R - 1 - k : NB - 1;
            if (k + NB - 1 < R) {
                __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0)
                __builtin_amdgcn_wave_barrier();
                issue((k + NB - 1) * m, ((kb + NB - 1) % NB) * hoff);
            }
            // younger than round k's fetch: the fetches of the rounds ahead, and the stores of the
            // rounds computed since it was issued (n outputs x 3 / 1 wave-level stores each)
            const uint32_t st = n * (FU ? 3u : 1u);
            wait_vm(ninst * ahead + st * (k < NB - 1 ? k : NB - 1));
        } else {
            __builtin_amdgcn_s_waitcnt(0);
        }
        hb = kb * hoff;
        kb = kb + 1 == NB ? 0u : kb + 1;
        __builtin_amdgcn_wave_barrier();
        if constexpr (L0 > 0) {
            // the shared levels of this round's (G x KS x m) staged groups of J chunks, in place
            // (every lane, active or not; one wave's LDS accesses complete in issue order)
            float4* curw = reinterpret_cast<float4*>(stg) + (hb >> 2);
            const uint32_t ng = (64u / LP) * KS * m;
            for (uint32_t gi = c.lane; gi < ng; gi += 64u) {
                const uint32_t g = gi % (64u / LP), q = gi / (64u / LP);
                float4 v[J];
#pragma unroll
                for (uint32_t j = 0; j < J; ++j)
                    v[j] = curw[stg_idx<LP>(q * J + j, g, per)];
#pragma unroll
                for (uint32_t l = 1; l <= L0; ++l)
#pragma unroll
                    for (uint32_t i = 0; i < (J >> l); ++i)
                        v[i] = f4_f(v[2 * i], v[2 * i + 1]);
#pragma unroll
                for (uint32_t j = 0; j < J0; ++j)
                    curw[stg_idx<LP>(q * J + j, g, per)] = v[j];
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (!w.act)
            continue;
#if defined(PCG_DEV_ABL_DEEP) && PCG_DEV_ABL_DEEP == 2 // dev ablation (wrong results): no arithmetic
        for (uint32_t uu = 0; uu < n; ++uu) {
            const uint32_t c2 = r + w.i * n + uu;
            d1.st(c2, make_float4(0.f, 0.f, 0.f, 0.f));
            if constexpr (FU) {
                d1.st(c2 + hq2, make_float4(0.f, 0.f, 0.f, 0.f));
                d2.st(c2, make_float4(0.f, 0.f, 0.f, 0.f));
            }
        }
        continue;
#endif
        const float4* cur = stg4 + (hb >> 2);
        for (uint32_t uu = 0; uu < n; ++uu) {
            const uint32_t u = w.i * n + uu, c2 = r + u;
            if (uu > 0 && (uu & 7u) == 0)
                words(c2);
            const uint32_t gs = 4u * (c2 & 7u);
            float4 x[KS];
#pragma unroll
            for (uint32_t k = 0; k < KS; ++k) {
                float4 v[J0];
#pragma unroll
                for (uint32_t j = 0; j < J0; ++j)
                    v[j] = cur[stg_idx<LP>((u * KS + k) * J + j, mg, per)];
#pragma unroll
                for (uint32_t l = L0 + 1; l <= (uint32_t)V; ++l)
#pragma unroll
                    for (uint32_t i = 0; i < (J >> l); ++i)
                        v[i] = ((RM >> (l - 1)) & 1) ? f4_g(v[2 * i], v[2 * i + 1], bw[k][J - (J >> (l - 1)) + i], gs)
                                                     : f4_f(v[2 * i], v[2 * i + 1]);
                x[k] = v[0];
            }
            const float4 y0 = OPC == OP_F ? f4_f(x[0], x[1]) : f4_g(x[0], x[1], lw[0], gs);
#if defined(PCG_DEV_ABL_DEEP) && PCG_DEV_ABL_DEEP == 3 // dev ablation (wrong results): no stores
            if (c.N != 0)
                continue;
#endif
            // (exactly 1 + 2 * FU store instructions per output chunk: the wait_vm count above
            // depends on it -- a conditional store here would let a round read stale LDS)
            d1.st(c2, y0);
            if constexpr (FU) {
                const float4 y1 = OPC == OP_F ? f4_f(x[2], x[3]) : f4_g(x[2], x[3], lw[1], gs);
                d1.st(c2 + hq2, y1);
                d2.st(c2, f4_f(y0, y1));
            }
        }
    }
#if PCG_STG_TAIL_DRAIN
    __builtin_amdgcn_s_waitcnt(0);
#else
    // every fetch has landed (the last round waited for its own); the LDS reads have completed
    // before later ops reuse the region -- the op's global stores drain behind the next ops
    // (same-wave accesses to one address stay ordered), not here
    __builtin_amdgcn_s_waitcnt(0xC07F); // lgkmcnt(0)
#endif
}

// the bits level l of a recomputed stage-(top-V) node at o reads: the left child of its
// level-l ancestor (l = 1: the root's left half; 2: D[top-1] / the row at the top-1 node;
// 3: D[top-2] / the row at the top-2 node) for the path in lane w.dl
template <int LP>
PCG_DEV void level_bits(const Ls<LP>& c, const Share& w, uint32_t o, DBits (&vb)[3])
{
    vb[0] = root_bits(c, w);
#pragma unroll
    for (uint32_t l = 2; l <= 3; ++l) {
        const uint32_t st = c.top + 1u - l;
        if constexpr (Ls<LP>::DB)
            vb[l - 1] = dbits(c, st, w.shr ? path_dlane(c, w.dl, st) : c.dlane(st));
        else
            vb[l - 1] = rowbits(c, w.dl, o & ~((1u << st) - 1u));
    }
}
// Run the staged op on the recomputed node of stage s = top-V at o (V = 2, or 3 for LP >= 16)
template <int OPC, bool FU, int LP>
PCG_DEV void ls_rootv_op(const Ls<LP>& c, GlSt d1, GlSt d2, const DBits& lb, uint32_t s, uint32_t o, const Share& w,
                         uint32_t m)
{
    DBits vb[3];
    level_bits(c, w, o, vb);
    const uint32_t V = c.top - s;
    // RM bit l-1: the level-l ancestor's right child holds the node
    uint32_t rm = 0;
    for (uint32_t l = 1; l <= V; ++l)
        rm |= ((o >> (c.top - l)) & 1u) << (l - 1);
    if (V == 2) {
        switch (rm) {
        case 0: ls_fgf_rootv<OPC, 2, 0, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 1: ls_fgf_rootv<OPC, 2, 1, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 2: ls_fgf_rootv<OPC, 2, 2, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        default: ls_fgf_rootv<OPC, 2, 3, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        }
        return;
    }
    if constexpr (LP >= 16) {
        switch (rm) {
        case 0: ls_fgf_rootv<OPC, 3, 0, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 1: ls_fgf_rootv<OPC, 3, 1, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 2: ls_fgf_rootv<OPC, 3, 2, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 3: ls_fgf_rootv<OPC, 3, 3, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 4: ls_fgf_rootv<OPC, 3, 4, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 5: ls_fgf_rootv<OPC, 3, 5, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        case 6: ls_fgf_rootv<OPC, 3, 6, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        default: ls_fgf_rootv<OPC, 3, 7, FU, LP>(c, d1, d2, lb, vb, s, w, m); break;
        }
    }
}

template <int OPC, int LP>
PCG_DEV void ls_fgf_op(Ls<LP>& c, uint32_t s, uint32_t o, uint32_t P)
{
    const uint32_t d = s - 1, e = s - 2;
    const bool rootc = s >= c.mt && s != c.top, left = o < (c.N >> 1), deep = rootc && s + 2u <= c.top;
    // (quarters / eighths: at most as many lanes per path as a staging round has output chunks,
    // so that the idle lanes of a codeword with P < LP paths share its staged rounds)
    const Share w = ls_share(c, P, s, deep ? PCG_DEEP_SHARE * 2u * ls_root_round(c, s, 1u, true) : 1u << (s - 4));
    const DBits lb = gbits(c, s, o, w.dl, w.bl);
    const uint32_t rm = ls_root_round(c, s, w.h, true);
    if (deep) { // a recomputed quarter / eighth: staged (its grandchild alpha[s-2] is global)
        if (rm) { // (always: sclls_layout plans virt >= 2 only when it stages)
            GlSt d1 = gl_st(c, d), d2 = gl_st(c, e);
            d1.lane = w.dl;
            d2.lane = w.dl;
            ls_rootv_op<OPC, true, LP>(c, d1, d2, lb, s, o, w, rm);
        }
        c.own(d);
        c.own(e);
        return;
    }
    const DBits rb = rootc && !left ? root_bits(c, w) : DBits{};
    auto run = [&](auto dst2) {
        GlSt d1 = gl_st(c, d);
        d1.lane = w.dl;
        dst2.lane = w.dl;
        if (s == c.top) {
            ls_fgf<OPC, LP>(ChSt{ c.y }, d1, dst2, lb, s, w);
        } else if (rm && left)
            ls_fgf_root<OPC, true, LP>(c, d1, dst2, lb, rb, s, w, rm);
        else if (rm)
            ls_fgf_root<OPC, false, LP>(c, d1, dst2, lb, rb, s, w, rm);
        else if (rootc && left)
            ls_fgf<OPC, LP>(RootSt<true>{ c.y, rb, c.N >> 3 }, d1, dst2, lb, s, w);
        else if (rootc)
            ls_fgf<OPC, LP>(RootSt<false>{ c.y, rb, c.N >> 3 }, d1, dst2, lb, s, w);
        else
            ls_fgf<OPC, LP>(gl_st(c, s), d1, dst2, lb, s, w);
    };
    if (e >= c.Sl)
        run(gl_st(c, e));
    else
        run(lds_st(c, e));
    c.own(d);
    c.own(e);
}

// ---- node results into the D buffers ----------------------------------------------------
// The 2^t result bits of the stage-t node at o go to the path's own lane: as its half of
// D[t+1] (the parent's children), or as D[top] for the root.  d_word(w, v) stores result
// word w (n = 2^t < 32: one call with the n bits, merged with the left half read from the
// slot for a right child); d_end copies the left half of a multi-word right child over
// from the slot, after every read of the op (the slot may be a lane that moves its own
// left half here) and sets the table.  Every store follows the wave-wide read of the same
// word, so lanes reading a column see it before its owner rewrites it.
template <int LP>
PCG_DEV uint32_t d_target(const Ls<LP>& c, uint32_t t) { return t == c.top ? t : t + 1u; }

// The word columns of one D stage (or of the LDS codeword region), LDS or global: distinct
// types so that each copy loop is compiled for its own address space.
struct DColL {
    lds_u32* b;
    PCG_DEV uint32_t ld(uint32_t w, uint32_t l) const { return b[(w << 6) + l]; }
    PCG_DEV void st(uint32_t w, uint32_t l, uint32_t v) const { b[(w << 6) + l] = v; }
};
struct DColG {
    gl_u32* b;
    PCG_DEV uint32_t ld(uint32_t w, uint32_t l) const
    {
        LS_GB(4, 0);
        return b[((uint64_t)w << 6) + l];
    }
    PCG_DEV void st(uint32_t w, uint32_t l, uint32_t v) const
    {
        LS_GB(4, 1);
        b[((uint64_t)w << 6) + l] = v;
    }
};
template <int LP, typename Fn>
PCG_DEV void with_d(const Ls<LP>& c, uint32_t s, Fn&& fn)
{
    const uint32_t o = ls_doff(s);
    if (s < c.Sb)
        fn(DColL{ c.dl + (o << 6) });
    else
        fn(DColG{ c.dg + ((uint64_t)(o - (1u << (c.Sb - 5u))) << 6) });
}
// words [0, nw) of lane sl's column -> this lane's column, 8 loads before their stores
template <typename Col>
PCG_DEV void d_copy(const Col& col, uint32_t nw, uint32_t sl, uint32_t lane)
{
    for (uint32_t w = 0; w < nw; w += 8) {
        uint32_t x[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u)
            if (w + u < nw)
                x[u] = col.ld(w + u, sl);
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u)
            if (w + u < nw)
                col.st(w + u, lane, x[u]);
    }
}

template <int LP>
PCG_DEV void d_word(const Ls<LP>& c, uint32_t t, uint32_t o, uint32_t w, uint32_t v)
{
    const uint32_t n = 1u << t, d = d_target(c, t);
    if (d == t || ((o >> t) & 1u) == 0u) { // the root, or a left child
        c.dst(d, w, v);
    } else if (n < 32u) {
        c.dst(d, 0, (c.dld(d, 0, c.dlane(d)) & ((1u << n) - 1u)) | (v << n));
    } else {
        c.dst(d, (n >> 5) + w, v);
    }
}
template <int LP>
PCG_DEV void d_end(Ls<LP>& c, uint32_t t, uint32_t o)
{
    const uint32_t n = 1u << t, d = d_target(c, t);
    if (d != t && ((o >> t) & 1u) && n >= 32u) {
        const uint32_t sl = c.dlane(d);
        with_d(c, d, [&](const auto& col) { d_copy(col, n >> 5, sl, c.lane); });
    }
    c.down(d);
}

// Combine (avx_float.h:188-197 on packed bits) of the stage-s node at o: its children
// D[s] = (l, r) give (l ^ r, r).  The root's codeword goes to the (now dead) LLR stage
// region of LDS when it fits there (fin): the output stage reads it word by word.
template <typename Src, typename Dst>
PCG_DEV void comb_words(const Src& S, uint32_t sl, const Dst& T, uint32_t ob, uint32_t nw, uint32_t lane)
{
    for (uint32_t w = 0; w < nw; w += 8) {
        uint32_t l[8], r[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u)
            if (w + u < nw) {
                l[u] = S.ld(w + u, sl);
                r[u] = S.ld(nw + w + u, sl);
            }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u)
            if (w + u < nw) {
                T.st(ob + w + u, lane, l[u] ^ r[u]);
                T.st(ob + nw + w + u, lane, r[u]);
            }
    }
}
template <int LP>
PCG_DEV void ls_comb(Ls<LP>& c, uint32_t s, uint32_t o, bool act)
{
    if constexpr (!Ls<LP>::DB) { // in the row: bit[o+i] ^= bit[o+h+i], i < h
        const uint32_t h = 1u << (s - 1);
        lds_u32* row = c.row();
        if (!act)
            return;
        if (h >= 32) {
            // (the left words are written, the right ones only read: 8 word pairs loaded per
            // batch before their stores, not one dependent LDS round trip per word)
            const uint32_t wl = o >> 5, wr = (o + h) >> 5, nw = h >> 5;
            for (uint32_t w = 0; w < nw; w += 8) {
                uint32_t l[8], r[8];
#pragma unroll
                for (uint32_t u = 0; u < 8; ++u)
                    if (w + u < nw) {
                        l[u] = row[(wl + w + u) << 6];
                        r[u] = row[(wr + w + u) << 6];
                    }
#pragma unroll
                for (uint32_t u = 0; u < 8; ++u)
                    if (w + u < nw)
                        row[(wl + w + u) << 6] = l[u] ^ r[u];
            }
        } else {
            const uint32_t sh = o & 31u, msk = ((1u << h) - 1u) << sh;
            lds_u32* w = row + ((o >> 5) << 6);
            *w ^= (*w >> h) & msk;
        }
        return;
    }
    const uint32_t h = 1u << (s - 1), sl = c.dlane(s);
    const bool root = s == c.top;
    if (root && h >= 32u && c.Sl > 3u + c.vlow && (h >> 4) <= (1u << c.Sl) - c.ab) {
        c.fin = true;
        if (act)
            with_d(c, s, [&](const auto& S) {
                comb_words(S, sl, DColL{ (lds_u32*)(c.lds + c.ly.alpha) }, 0u, h >> 5, c.lane);
            });
        return;
    }
    if (!act)
        return;
    if (h < 32u) { // s = 4, 5: one word
        const uint32_t x = c.dld(s, 0, sl), m = (1u << h) - 1u;
        d_word(c, s, o, 0, ((x ^ (x >> h)) & m) | (x & (m << h)));
    } else {
        const uint32_t d = d_target(c, s), ob = !root && ((o >> s) & 1u) ? h >> 4 : 0u;
        with_d(c, s, [&](const auto& S) {
            with_d(c, d, [&](const auto& T) { comb_words(S, sl, T, ob, h >> 5, c.lane); });
        });
    }
    d_end(c, s, o);
}

// Rate-0: the all-zero estimate.
template <int LP>
PCG_DEV void ls_clear(Ls<LP>& c, uint32_t t, uint32_t o)
{
    const uint32_t n = 1u << t;
    if constexpr (!Ls<LP>::DB) { // bits [o, o+n) of the row
        lds_u32* row = c.row();
        if (n >= 32) {
            for (uint32_t w = o >> 5; w < (o + n) >> 5; ++w)
                row[w << 6] = 0u;
        } else {
            row[(o >> 5) << 6] &= ~(((1u << n) - 1u) << (o & 31u));
        }
        return;
    }
    for (uint32_t w = 0; w < (n >= 32u ? n >> 5 : 1u); ++w)
        d_word(c, t, o, w, 0u);
    d_end(c, t, o);
}

// ---- Rate-0 leaf, n >= 8 (scl_avx_float.cpp:316-337) ----------------------------------
// metric += reduce_add_ps(sum over 8-float vectors of min(llr, +0)): lane j of the AVX
// accumulator takes elements j, j+8, ... from +0, then ((((((a0+a1)+a2)+a3)+a4)+a5)+a6)+a7.
template <int LP, typename Src>
PCG_DEV void ls_r0(Ls<LP>& c, Src src, uint32_t s, uint32_t o, bool act)
{
    const uint32_t nq = 1u << (s - 2);
    const uint32_t sl = s == c.top ? 0u : c.src_lane(s);
    if (!act)
        return;
    float acc[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
    constexpr int U = Pre<Src>::U; // even
    stream<U>(src, nq, sl, [&](const float4 (&x)[U], uint32_t c0, uint32_t valid) {
#pragma unroll
        for (int u = 0; u < U; u += 2) {
            if ((uint32_t)u < valid) { // chunks come in pairs (nq, valid even): one 8-float vector
                const float4 a = x[u], b = x[u + 1];
                acc[0] = acc[0] + minps(a.x, 0.0f);
                acc[1] = acc[1] + minps(a.y, 0.0f);
                acc[2] = acc[2] + minps(a.z, 0.0f);
                acc[3] = acc[3] + minps(a.w, 0.0f);
                acc[4] = acc[4] + minps(b.x, 0.0f);
                acc[5] = acc[5] + minps(b.y, 0.0f);
                acc[6] = acc[6] + minps(b.z, 0.0f);
                acc[7] = acc[7] + minps(b.w, 0.0f);
            }
        }
    });
    float r = acc[0];
#pragma unroll
    for (int j = 1; j < 8; ++j)
        r = r + acc[j];
    c.m = c.m + r;
    ls_clear(c, s, o);
}

// ---- weak positions: findWeakLlrs(idx, |llr|, n, kk) (arrayfuncs.h:209-231) ------------
// Exact selection passes with the reference's swaps: pass t takes the first minimum
// of positions >= t; the element it displaces is tracked in a <= 4 entry overlay.
// Results T[t] (value) and I[t] (original index) for t < kk, and the XOR of the n
// sign bits.  n >= 16 (size-8 leaves use the register version).
template <int LP, typename Src>
PCG_DEV void ls_weak(const Ls<LP>& c, Src src, uint32_t sl, uint32_t n, uint32_t kk, float (&T)[4],
                     uint32_t (&I)[4], uint32_t& par)
{
    const uint32_t nq = n >> 2;
    par = 0;
    uint32_t ovp[4] = { ~0u, ~0u, ~0u, ~0u }, ovi[4] = { 0, 0, 0, 0 };
    float ovv[4] = { 0, 0, 0, 0 };
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t) {
        T[t] = 0.0f;
        I[t] = t;
        if (t >= kk)
            continue;
        // scan raw positions > t that are not in the overlay; the overlay and
        // position t itself are merged afterwards by (value, position)
        float bv = __builtin_inff();
        uint32_t bi = ~0u;
        for (uint32_t q = 0; q < nq; ++q) {
            const float4 x = src.ld(q, sl);
            if (t == 0)
                par ^= fbits(x.x) ^ fbits(x.y) ^ fbits(x.z) ^ fbits(x.w);
            const float xv[4] = { x.x, x.y, x.z, x.w };
#pragma unroll
            for (uint32_t e = 0; e < 4; ++e) {
                const uint32_t i = 4u * q + e;
                bool ok = i > t;
#pragma unroll
                for (uint32_t r = 0; r < 4; ++r)
                    if (r < t)
                        ok = ok && i != ovp[r];
                const float v = fabs_(xv[e]);
                if (ok && (bi == ~0u || v < bv)) {
                    bv = v;
                    bi = i;
                }
            }
        }
        // the element currently at position t
        float vt;
        {
            const float4 x = src.ld(t >> 2, sl);
            const uint32_t e = t & 3u;
            vt = fabs_(e == 0 ? x.x : e == 1 ? x.y : e == 2 ? x.z : x.w);
        }
        uint32_t it = t;
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r)
            if (r < t && ovp[r] == t) {
                vt = ovv[r];
                it = ovi[r];
            }
        // overlay entries at positions > t compete by (value, position)
#pragma unroll
        for (uint32_t r = 0; r < 4; ++r) {
            if (r < t && ovp[r] != ~0u && ovp[r] > t &&
                (bi == ~0u || ovv[r] < bv || (ovv[r] == bv && ovp[r] < bi))) {
                bv = ovv[r];
                bi = ovp[r];
            }
        }
        // position t itself wins ties (it comes first)
        uint32_t bo;
        if (bi == ~0u || !(bv < vt)) {
            bv = vt;
            bi = t;
            bo = it;
        } else {
            bo = bi;
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r)
                if (r < t && ovp[r] == bi)
                    bo = ovi[r];
        }
        T[t] = bv;
        I[t] = bo;
        if (bi != t) { // the element at position t moves to position bi
            bool placed = false;
#pragma unroll
            for (uint32_t r = 0; r < 4; ++r)
                if (r < t && ovp[r] == bi) {
                    ovv[r] = vt;
                    ovi[r] = it;
                    placed = true;
                }
            if (!placed) {
                ovp[t] = bi;
                ovv[t] = vt;
                ovi[t] = it;
            }
        }
    }
}

// One streaming pass for the same result when it is unambiguous: the lim+1 smallest
// |llr| (stable insertion) with their indices, and the parity.  Pass t of the
// reference picks the (t+1)-th smallest; only equal values among the first lim+1 make
// its swap order observable -- then *tie is set and ls_weak runs instead.
template <int LP, typename Src>
PCG_DEV void weak_fast(Src src, uint32_t sl, uint32_t n, uint32_t kk, float (&T)[4], uint32_t (&I)[4],
                       uint32_t& par, bool& tie)
{
    float sv[5];
    uint32_t si[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        sv[j] = __builtin_inff();
        si[j] = ~0u;
    }
    uint32_t px = 0;
    const bool r1 = kk == 2u; // keep 3 entries for Rate-1, 5 for SPC
    constexpr int U = Pre<Src>::U;
    stream<U>(src, n >> 2, sl, [&](const float4 (&x)[U], uint32_t c0, uint32_t valid) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if ((uint32_t)u < valid) {
                const float xv[4] = { x[u].x, x[u].y, x[u].z, x[u].w };
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    px ^= fbits(xv[e]);
                    float v = fabs_(xv[e]);
                    uint32_t i = 4u * (c0 + u) + e;
#pragma unroll
                    for (int j = 0; j < 5; ++j) {
                        if (j < 3 || !r1) {
                            const bool lt = v < sv[j];
                            const float tv = sv[j];
                            const uint32_t ti = si[j];
                            sv[j] = lt ? v : tv;
                            si[j] = lt ? i : ti;
                            v = lt ? tv : v;
                            i = lt ? ti : i;
                        }
                    }
                }
            }
        }
    });
    par = px;
    bool t = false;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if ((uint32_t)j < kk)
            t = t || sv[j] == sv[j + 1];
    tie = t;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        T[j] = (uint32_t)j < kk ? sv[j] : 0.0f;
        I[j] = (uint32_t)j < kk ? si[j] : (uint32_t)j;
    }
}

// The same pass on 32-bit keys (PCG_WEAK_K32): the |llr| bits with their low log2(n) bits
// replaced by the element index, kept by a v_min_u32 / v_max_u32 insertion chain (two ops per
// kept entry and element instead of a compare and four selects).  The keys order the elements
// as (value, index) does except among values that agree above those low bits; so when two of
// the first kk+1 kept keys agree there, false is returned and the float pass runs.  The kept
// entries' exact values are re-read (kk loads).
#ifndef PCG_WEAK_K32
#define PCG_WEAK_K32 1
#endif
#ifndef PCG_WEAK_K32_LP
#define PCG_WEAK_K32_LP 32
#endif
template <int LP, int KEEP, typename Src>
PCG_DEV bool weak_keys(Src src, uint32_t sl, uint32_t n, uint32_t kk, float (&T)[4], uint32_t (&I)[4],
                       uint32_t& par)
{
    const uint32_t cb = (uint32_t)__builtin_ctz(n), cm = (1u << cb) - 1u;
    uint32_t sk[KEEP];
#pragma unroll
    for (int j = 0; j < KEEP; ++j)
        sk[j] = ~0u;
    uint32_t px = 0;
    constexpr int U = Pre<Src>::U;
    stream<U>(src, n >> 2, sl, [&](const float4 (&x)[U], uint32_t c0, uint32_t valid) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if ((uint32_t)u < valid) {
                const uint32_t xb[4] = { fbits(x[u].x), fbits(x[u].y), fbits(x[u].z), fbits(x[u].w) };
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    px ^= xb[e];
                    uint32_t key = (xb[e] & 0x7fffffffu & ~cm) | (4u * (c0 + u) + e);
#pragma unroll
                    for (int j = 0; j < KEEP; ++j) {
                        const uint32_t lo = key < sk[j] ? key : sk[j];
                        key = umax32(key, sk[j]);
                        sk[j] = lo;
                    }
                }
            }
        }
    });
    par = px;
    bool near = false;
#pragma unroll
    for (int j = 0; j + 1 < KEEP; ++j)
        if ((uint32_t)j < kk)
            near = near || (sk[j] >> cb) == (sk[j + 1] >> cb);
    if (near)
        return false;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t i = sk[j < KEEP ? j : 0] & cm;
        if ((uint32_t)j < kk) {
            const float4 v = src.ld(i >> 2, sl);
            const uint32_t e = i & 3u;
            T[j] = fabs_(e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w);
            I[j] = i;
        } else {
            T[j] = 0.0f;
            I[j] = (uint32_t)j;
        }
    }
    return true;
}

// Register version for n == 8 (and the same selection passes as ls_weak).
PCG_DEV void weak8(const float (&v)[8], uint32_t kk, float (&T4)[4], uint32_t (&I4)[4], uint32_t& par)
{
    float T[8];
    uint32_t I[8];
    par = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        T[j] = fabs_(v[j]);
        I[j] = (uint32_t)j;
        par ^= fbits(v[j]);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (t < (int)kk) {
            float bv = T[t];
            uint32_t b = (uint32_t)t;
#pragma unroll
            for (int j = t + 1; j < 8; ++j) {
                const bool better = T[j] < bv;
                bv = better ? T[j] : bv;
                b = better ? (uint32_t)j : b;
            }
            const uint32_t tv = fbits(T[t]), ti = I[t];
            uint32_t bi = I[t];
#pragma unroll
            for (int j = t + 1; j < 8; ++j) {
                const uint32_t mj = 0u - (uint32_t)(b == (uint32_t)j);
                bi = (I[j] & mj) | (bi & ~mj);
                T[j] = ubits((tv & mj) | (fbits(T[j]) & ~mj));
                I[j] = (ti & mj) | (I[j] & ~mj);
            }
            T[t] = bv;
            I[t] = bi;
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        T4[t] = T[t];
        I4[t] = I[t];
    }
}

// Candidate metrics of Rate-1 (:365-379, 4 candidates) and SPC (:511-585, 8).
PCG_DEV void r1_spc_cands(uint32_t code, float m, const float (&T)[4], uint32_t par, float (&cv)[8])
{
    if (code == OP_S_R1) {
        cv[0] = m;
        cv[1] = m - T[0];
        cv[2] = m - T[1];
        cv[3] = m - T[0] - T[1];
        cv[4] = cv[5] = cv[6] = cv[7] = 0.0f;
        return;
    }
    float mm = m, pinv = 1.0f;
    if (par & 0x80000000u) { // odd parity: the reference charges T0 up front
        pinv = 0.0f;
        mm -= T[0];
    }
    cv[0] = mm;
    cv[1] = mm - pinv * T[0] - T[1];
    cv[2] = mm - pinv * T[0] - T[2];
    cv[3] = mm - pinv * T[0] - T[3];
    cv[4] = mm - T[1] - T[2];
    cv[5] = mm - T[1] - T[3];
    cv[6] = mm - T[2] - T[3];
    cv[7] = mm - pinv * T[0] - T[1] - T[2] - T[3];
}

// flip mask over the 4 weak indices for candidate j (nibble tables, see scl_kernel.hip):
// R1 {}, {i0}, {i1}, {i0,i1}; SPC even {}, {0,1}, {0,2}, {0,3}, {1,2}, {1,3}, {2,3},
// {0,1,2,3}; SPC odd {0}, {1}, {2}, {3}, {0,1,2}, {0,1,3}, {0,2,3}, {1,2,3}.
PCG_DEV uint32_t ls_flip_sel(uint32_t code, uint32_t j, uint32_t oddpar)
{
    const uint32_t tab = code == OP_S_R1 ? 0x3210u : oddpar ? 0xEDB78421u : 0xFCA69530u;
    return (tab >> (4 * j)) & 0xFu;
}

// ---- path selection over the group ---------------------------------------------------
// Candidates cv[0..K) of every active path (p < P), enumerated as e = p*K + j like the
// reference's metric array.  Survivor q < np (descending metric, the order
// simplePartialSortDescending leaves) is delivered to lane q of the group as
// (val, src path, j).  Fast path: local sorting network + LP-lane merge rounds; if
// any adjacent pair among the first lim+1 selected values is equal (the only case in
// which the swap order shows), every group re-runs the literal selection sort.
// Candidates travel as 64-bit keys: the float's order-preserving integer image above
// ~code (code = path << 3 | j), so one unsigned compare orders by value and makes
// every key unique.  -0 and +0 get different keys; they compare equal as floats, so
// such a pair is caught by the tie test like any other equal pair.
PCG_DEV uint32_t ord_of(float v)
{
    const uint32_t u = fbits(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
PCG_DEV float val_of(uint32_t o) { return ubits((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o); }

PCG_DEV void cx_desc(uint64_t (&k)[8], int a, int b)
{
    const uint64_t ka = k[a], kb = k[b];
    const bool sw = kb > ka;
    k[a] = sw ? kb : ka;
    k[b] = sw ? ka : kb;
}

// The candidate lists come out of r1_spc_cands / st_cands8 almost sorted: with the weak
// magnitudes ascending (T0 <= T1 <= T2 <= T3, findWeakLlrs' pass order) and fp subtraction
// monotone in both operands, Rate-1 gives c0 >= c1 >= c2 >= c3 and SPC (either parity)
// c0 >= c1 >= c2 >= {c3, c4} >= c5 >= c6 >= c7 -- only c3 / c4 are unordered; Repetition's
// two candidates are.  Among float-equal values the structural order puts the lower
// candidate index first, which is the key order too (a -0 below a +0 cannot follow from
// these subtractions), so one compare-exchange of keys sorts every list.
template <int K>
PCG_DEV void local_order(uint64_t (&k)[8])
{
    if constexpr (K == 2)
        cx_desc(k, 0, 1);
    else if constexpr (K == 8)
        cx_desc(k, 3, 4);
}

template <int K>
PCG_DEV void local_sort(uint64_t (&k)[8])
{
    if constexpr (K == 2) {
        cx_desc(k, 0, 1);
    } else if constexpr (K == 4) {
        cx_desc(k, 0, 1); cx_desc(k, 2, 3);
        cx_desc(k, 0, 2); cx_desc(k, 1, 3);
        cx_desc(k, 1, 2);
    } else {
        // 19-comparator network for 8 inputs
        cx_desc(k, 0, 2); cx_desc(k, 1, 3); cx_desc(k, 4, 6); cx_desc(k, 5, 7);
        cx_desc(k, 0, 4); cx_desc(k, 1, 5); cx_desc(k, 2, 6); cx_desc(k, 3, 7);
        cx_desc(k, 0, 1); cx_desc(k, 2, 3); cx_desc(k, 4, 5); cx_desc(k, 6, 7);
        cx_desc(k, 2, 4); cx_desc(k, 3, 5);
        cx_desc(k, 1, 4); cx_desc(k, 3, 6);
        cx_desc(k, 1, 2); cx_desc(k, 3, 4); cx_desc(k, 5, 6);
    }
}

template <int J>
PCG_DEV void kmax_step(uint64_t& k)
{
    const uint32_t lo = xpartner<J>((uint32_t)k), hi = xpartner<J>((uint32_t)(k >> 32));
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    k = o > k ? o : k;
}

template <int LP>
PCG_DEV void grp_kmax(uint64_t& k)
{
    if constexpr (LP > 1) kmax_step<1>(k);
    if constexpr (LP > 2) kmax_step<2>(k);
    if constexpr (LP > 4) kmax_step<4>(k);
    if constexpr (LP > 8) kmax_step<8>(k);
    if constexpr (LP > 16) kmax_step<16>(k);
    if constexpr (LP > 32) kmax_step<32>(k);
}

// ---- bitonic variant of the merge rounds (LP >= PCG_SEL_BITONIC_LP) ----------------------
// The keys are unique, so any exact sort yields the merge rounds' order.  Lane p holds
// elements p*K .. p*K+K-1 of the group's sequence (its locally sorted run); log2(LP)
// bitonic merge levels double the sorted runs: a mirror stage (lane p ^ (2B-1),
// register K-1-j) then half-cleaners (exact xor partners, then in-register pairs).
// Every stage is K independent compare-exchanges through DPP / permlane -- no
// dependent chain of np+1 group reductions.
#ifndef PCG_SEL_BITONIC_LP
#define PCG_SEL_BITONIC_LP 16
#endif
#ifndef PCG_SEL_BITONIC_K // also for short candidate lists at any LP
#define PCG_SEL_BITONIC_K 4 // K = 2 / 4 lists at LP = 8: 1.87e7 -> 1.93e7 cw/s (r02z sweep)
#endif
template <int B> // lane i <- lane i ^ (B-1) within aligned blocks of B lanes
PCG_DEV uint32_t mirror_lane(uint32_t v)
{
    if constexpr (B == 2)
        return xpartner<1>(v);
    else if constexpr (B == 4)
        return xpartner<2>(xpartner<1>(v)); // i ^ 3
    else if constexpr (B == 8)
        return bfly<4>(v); // row_half_mirror
    else if constexpr (B == 16)
        return bfly<8>(v); // row_mirror
    else
        return xpartner<16>(bfly<8>(v)); // B == 32: 31 - i
}
template <int B>
PCG_DEV uint64_t mirror64(uint64_t k)
{
    return ((uint64_t)mirror_lane<B>((uint32_t)(k >> 32)) << 32) | mirror_lane<B>((uint32_t)k);
}
template <int J>
PCG_DEV uint64_t xpart64(uint64_t k)
{
    return ((uint64_t)xpartner<J>((uint32_t)(k >> 32)) << 32) | xpartner<J>((uint32_t)k);
}
PCG_DEV uint64_t kmax(uint64_t a, uint64_t b) { return b > a ? b : a; }
PCG_DEV uint64_t kmin(uint64_t a, uint64_t b) { return b > a ? a : b; }
// low ? max(k, o) : min(k, o): one compare, the lane's direction applied to its mask (SALU),
// one select per dword -- instead of both extrema and a third select (equal keys: either)
PCG_DEV uint64_t kdir(uint64_t k, uint64_t o, bool low) { return (o > k) == low ? o : k; }
PCG_DEV uint32_t kdir32(uint32_t k, uint32_t o, bool low) { return (o > k) == low ? o : k; }

template <int K, int D> // half-cleaner stages at lane distances D, D/2, .., 1
PCG_DEV void bit_lanes(uint64_t (&k)[8], uint32_t p)
{
    if constexpr (D >= 1) {
        const bool low = (p & D) == 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            k[j] = kdir(k[j], xpart64<D>(k[j]), low);
        }
        bit_lanes<K, D / 2>(k, p);
    }
}
template <int K, int D> // in-register half-cleaners at element distances D, .., 1
PCG_DEV void bit_regs(uint64_t (&k)[8])
{
    if constexpr (D >= 1) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            if ((j & D) == 0)
                cx_desc(k, j, j | D);
        bit_regs<K, D / 2>(k);
    }
}
template <int LP, int K, int B> // merge runs of B lanes into runs of 2B lanes
PCG_DEV void bit_level(uint64_t (&k)[8], uint32_t p)
{
    if constexpr (B < LP) {
        const bool low = (p & B) == 0;
        uint64_t t[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            t[j] = mirror64<2 * B>(k[K - 1 - j]);
#pragma unroll
        for (int j = 0; j < K; ++j)
            k[j] = kdir(k[j], t[j], low);
        bit_lanes<K, B / 2>(k, p);
        bit_regs<K, K / 2>(k);
        bit_level<LP, K, 2 * B>(k, p);
    }
}

// Float equality of two order images (+0 and -0 compare equal) in integer arithmetic
// (a float compare here crashes this compiler's instruction selection).
PCG_DEV bool ord_eq(uint32_t a, uint32_t b)
{
    const uint32_t za = a == 0x7fffffffu ? 0x80000000u : a, zb = b == 0x7fffffffu ? 0x80000000u : b;
    return za == zb;
}

// Survivor p (< np) of the sorted group sequence and the tie test over its first R.
template <int LP, int K>
PCG_DEV uint64_t bit_pick(const uint64_t (&k)[8], uint32_t p, uint32_t gb, uint32_t np, uint32_t R, bool& tie)
{
    tie = false;
#pragma unroll
    for (int j = 0; j + 1 < K; ++j)
        if (p * K + j + 1 < R)
            tie = tie | (ord_eq((uint32_t)(k[j] >> 32), (uint32_t)(k[j + 1] >> 32)));
    const uint32_t nxt = shfl((uint32_t)(k[0] >> 32), (int)(gb | ((p + 1) & (LP - 1))));
    if (p + 1 < LP && p * K + K < R)
        tie = tie | ord_eq((uint32_t)(k[K - 1] >> 32), nxt);
    const int sl = (int)(gb | (p / K));
    uint64_t mine = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t lo = shfl((uint32_t)k[j], sl), hi = shfl((uint32_t)(k[j] >> 32), sl);
        if ((uint32_t)j == p % K)
            mine = ((uint64_t)hi << 32) | lo;
    }
    return p < np ? mine : 0ull;
}

// ---- 32-bit keys (PCG_SEL_K32) ---------------------------------------------------------
// The bitonic merge on one dword per candidate: the value's order image (+0 and -0 mapped to
// one image) with its low CB = 3 + log2(LP) bits replaced by ~(path << 3 | j), so a compare-
// exchange is a v_max_u32 / v_min_u32 on a DPP operand instead of a 64-bit compare and four
// selects.  These keys order the candidates exactly as the 64-bit keys do, except among
// candidates whose values agree above the CB low bits ("near ties", relative 2^-(23-CB): a
// class of equal truncated values comes out contiguous, in any order).  So the first R
// selected keys are checked pairwise: a near tie anywhere -- exact ties and +-0 included -- sends
// the wave to the exact 64-bit sort (and from there, on a true tie, to the literal selection);
// otherwise the order, the survivors and the tie test are the 64-bit sort's.  Measured on
// config 3 with the selection ablated: selection is 27 % of the list kernel's VALU
// instructions (profiles/r04e_scl8_ablation.txt).
#ifndef PCG_SEL_K32
#define PCG_SEL_K32 1
#endif
#ifndef PCG_SEL_K32_LP
#define PCG_SEL_K32_LP 8 // widest list on the 32-bit keys
#endif
PCG_DEV uint32_t ordz(float v)
{
    const uint32_t o = ord_of(v);
    return o == 0x7fffffffu ? 0x80000000u : o; // -0 -> the image of +0
}
PCG_DEV void cx32(uint32_t (&k)[8], int a, int b)
{
    const uint32_t ka = k[a], kb = k[b];
    k[a] = umax32(ka, kb);
    k[b] = ka > kb ? kb : ka;
}
template <int K>
PCG_DEV void local_order32(uint32_t (&k)[8])
{
    if constexpr (K == 2)
        cx32(k, 0, 1);
    else if constexpr (K == 8)
        cx32(k, 3, 4);
}
template <int K, int D>
PCG_DEV void bit_lanes32(uint32_t (&k)[8], uint32_t p)
{
    if constexpr (D >= 1) {
        const bool low = (p & D) == 0;
#pragma unroll
        for (int j = 0; j < K; ++j) {
            k[j] = kdir32(k[j], xpartner<D>(k[j]), low);
        }
        bit_lanes32<K, D / 2>(k, p);
    }
}
template <int K, int D>
PCG_DEV void bit_regs32(uint32_t (&k)[8])
{
    if constexpr (D >= 1) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            if ((j & D) == 0)
                cx32(k, j, j | D);
        bit_regs32<K, D / 2>(k);
    }
}
template <int LP, int K, int B>
PCG_DEV void bit_level32(uint32_t (&k)[8], uint32_t p)
{
    if constexpr (B < LP) {
        const bool low = (p & B) == 0;
        uint32_t t[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            t[j] = mirror_lane<2 * B>(k[K - 1 - j]);
#pragma unroll
        for (int j = 0; j < K; ++j)
            k[j] = kdir32(k[j], t[j], low);
        bit_lanes32<K, B / 2>(k, p);
        bit_regs32<K, K / 2>(k);
        bit_level32<LP, K, 2 * B>(k, p);
    }
}
// Code bits of a candidate: its path (log2 LP bits) and its index in a K-candidate list
// (log2 K: 1 for Repetition, 2 for Rate-1, 3 for SPC) -- the fewer, the more value bits the
// key keeps and the rarer the near ties (LP = 32, K = 2: 26 value bits, not 24)
template <int K>
constexpr uint32_t k32_lk()
{
    return K <= 2 ? 1u : K <= 4 ? 2u : 3u;
}
template <int LP, int K = 8>
constexpr uint32_t k32_cb()
{
    return (LP <= 2 ? 1u : LP <= 4 ? 2u : LP <= 8 ? 3u : LP <= 16 ? 4u : 5u) + k32_lk<K>();
}
// Top-8 of an 8-lane group's 64 keys (LP = 8, K = 8: SPC leaves, np <= 8): instead of sorting
// all 64, three butterfly levels each merge the lane's sorted 8 with its partner's into the top
// 8 of both (max against the partner's run reversed: a bitonic sequence, then three in-register
// half-cleaners), after which every lane of the group holds the group's sorted top 8 -- 3 x 20
// compare-exchanges instead of the full bitonic sort's 84, and each survivor reads its key from
// its own registers (no cross-lane extraction).  The first non-survivor (R = np + 1 = 9, for the
// tie test) is the group maximum of the keys below the 8th.  Same keys, same order: the result
// and the near-tie test are the full sort's.
#ifndef PCG_SEL_TOP8
#define PCG_SEL_TOP8 1
#endif
template <int D>
PCG_DEV void top8_level(uint32_t (&q)[8])
{
    uint32_t t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        t[j] = bfly<D>(q[7 - j]);
#pragma unroll
    for (int j = 0; j < 8; ++j)
        q[j] = umax32(q[j], t[j]);
    bit_regs32<8, 4>(q);
}
template <int LP>
PCG_DEV bool k32_top8(const Ls<LP>& c, const float (&cv)[8], uint32_t P, uint32_t np, uint32_t R, float& val,
                      uint32_t& src, uint32_t& jsel)
{
    constexpr uint32_t CB = k32_cb<LP>(), cm = (1u << CB) - 1u;
    const bool act = c.p < P;
    auto key = [&](int j) { return act ? ((ordz(cv[j]) & ~cm) | (~((c.p << 3) | (uint32_t)j) & cm)) : 0u; };
    uint32_t q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        q[j] = key(j);
    local_order32<8>(q);
    top8_level<1>(q);
    top8_level<2>(q);
    top8_level<4>(q);
    // near ties among the first R (<= 9) of the group's sequence: q[0..7], then the 9th
    bool near = false;
#pragma unroll
    for (int j = 0; j + 1 < 8; ++j)
        if ((uint32_t)j + 1u < R)
            near = near | ((q[j] >> CB) == (q[j + 1] >> CB));
    if (R > 8u) {
        uint32_t m9 = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint32_t k = key(j);
            m9 = umax32(m9, k < q[7] ? k : 0u);
        }
        m9 = umax32(m9, bfly<1>(m9));
        m9 = umax32(m9, bfly<2>(m9));
        m9 = umax32(m9, bfly<4>(m9));
        near = near | ((q[7] >> CB) == (m9 >> CB));
    }
    if (ballot(near) != 0ull)
        return false;
    uint32_t mk = q[0];
#pragma unroll
    for (int j = 1; j < 8; ++j)
        mk = c.p == (uint32_t)j ? q[j] : mk;
    const uint32_t code = ~mk & cm;
    src = code >> 3;
    jsel = code & 7u;
    float vv = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float x = shfl(cv[j], (int)(c.gb | src));
        if ((uint32_t)j == jsel)
            vv = x;
    }
    val = vv;
    (void)np;
    return true;
}

// Selection on 32-bit keys: true and (val, src, jsel) when no group has a near tie among its
// first R selected keys, else false (the caller runs the exact sort).
template <int LP, int K>
PCG_DEV bool k32_select(const Ls<LP>& c, const float (&cv)[8], uint32_t P, uint32_t np, uint32_t R, float& val,
                        uint32_t& src, uint32_t& jsel)
{
    if constexpr (PCG_SEL_TOP8 && LP == 8 && K == 8)
        return k32_top8<LP>(c, cv, P, np, R, val, src, jsel);
    constexpr uint32_t CB = k32_cb<LP, K>(), cm = (1u << CB) - 1u, LK = k32_lk<K>();
    const bool act = c.p < P;
    uint32_t q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        q[j] = (act && j < K) ? ((ordz(cv[j]) & ~cm) | (~((c.p << LK) | (uint32_t)j) & cm)) : 0u;
    local_order32<K>(q);
    bit_level32<LP, K, 1>(q, c.p);
    bool near = false;
#pragma unroll
    for (int j = 0; j + 1 < K; ++j)
        if (c.p * K + j + 1 < R)
            near = near | ((q[j] >> CB) == (q[j + 1] >> CB));
    const uint32_t nxt = shfl(q[0], (int)(c.gb | ((c.p + 1) & (LP - 1))));
    if (c.p + 1 < LP && c.p * K + K < R)
        near = near | ((q[K - 1] >> CB) == (nxt >> CB));
    if (ballot(near) != 0ull)
        return false;
    const int sl = (int)(c.gb | (c.p / K));
    uint32_t mk = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const uint32_t x = shfl(q[j], sl);
        if ((uint32_t)j == c.p % K)
            mk = x;
    }
    const uint32_t code = ~mk & cm;
    src = code >> LK;
    jsel = code & ((1u << LK) - 1u);
    // the exact value of the candidate, from its path's lane
    float vv = 0.0f;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const float x = shfl(cv[j], (int)(c.gb | src));
        if ((uint32_t)j == jsel)
            vv = x;
    }
    val = vv;
    return true;
}

// ---- value merge rounds (PCG_SEL_VMERGE) ------------------------------------------------
// The same selection on 32-bit order images of the values alone: round r takes the group
// maximum of the lanes' heads (DPP butterflies of v_max_u32), the lowest lane holding it pops
// its head, and slot r records (value, lane); the popped position of slot r's candidate is the
// number of rounds its lane won before r.  Without a tie among the first R selected values
// (equal adjacent values, or two lanes holding the maximum in one round -- then the literal
// selection runs, as for the keyed variants) every round's maximum is unique, so the result is
// the keyed merge's.  The lists come in locally ordered (local_order: for K = 8 positions 3 / 4,
// for K = 2 positions 0 / 1 may have been exchanged), which maps a popped position back to the
// candidate index.
#ifndef PCG_SEL_VMERGE
#define PCG_SEL_VMERGE 0
#endif
template <int LP>
PCG_DEV uint32_t grp_umax(uint32_t v)
{
    if constexpr (LP > 1) v = umax32(v, bfly<1>(v));
    if constexpr (LP > 2) v = umax32(v, bfly<2>(v));
    if constexpr (LP > 4) v = umax32(v, bfly<4>(v));
    if constexpr (LP > 8) v = umax32(v, bfly<8>(v));
    if constexpr (LP > 16) v = umax32(v, bfly<16>(v));
    if constexpr (LP > 32) v = umax32(v, bfly<32>(v));
    return v;
}
template <int LP, int K>
PCG_DEV void vmerge_select(const Ls<LP>& c, const uint64_t (&k)[8], uint32_t P, uint32_t np, uint32_t R, float& val,
                           uint32_t& src, uint32_t& jsel, bool& tie)
{
    uint32_t hv[K];
    uint32_t swp = 0; // the local order exchanged a pair of positions
#pragma unroll
    for (int j = 0; j < K; ++j) {
        hv[j] = (uint32_t)(k[j] >> 32);
        const uint32_t jj = ~(uint32_t)k[j] & 7u; // candidate index of position j
        swp |= jj != (uint32_t)j ? 1u : 0u;
    }
    const uint64_t gmask = LP == 64 ? ~0ull : ((1ull << LP) - 1ull);
    uint32_t won = 0, mh = 0, mw = c.p, prevh = 0;
    bool t = false;
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t h = grp_umax<LP>(hv[0]);
        const uint64_t at = ballot(hv[0] == h);
        const uint32_t gm = (uint32_t)((at >> c.gb) & gmask);
        const uint32_t w = (uint32_t)__builtin_ctz(gm);
        t = t | ((gm & (gm - 1u)) != 0u) | ((r > 0) & ord_eq(h, prevh));
        prevh = h;
        const bool mine = c.p == r;
        mh = mine ? h : mh;
        mw = mine ? w : mw;
        const bool win = c.p == w;
        won |= (win && r < 32u) ? 1u << r : 0u;
#pragma unroll
        for (int j = 0; j + 1 < K; ++j)
            hv[j] = win ? hv[j + 1] : hv[j];
        hv[K - 1] = win ? 0u : hv[K - 1];
    }
    tie = t;
    const int sl = (int)(c.gb | mw);
    const uint32_t wsrc = shfl(won, sl), ssrc = shfl(swp, sl);
    uint32_t pos = (uint32_t)__builtin_popcount(wsrc & ((1u << (c.p & 31u)) - 1u));
    if (ssrc && K == 8 && (pos == 3u || pos == 4u))
        pos ^= 7u;
    if (ssrc && K == 2)
        pos ^= 1u;
    val = val_of(mh);
    src = mw;
    jsel = pos;
}

template <int LP, int K>
PCG_DEV void ls_select(const Ls<LP>& c, const float (&cv)[8], uint32_t P, uint32_t np, float& val, uint32_t& src,
                       uint32_t& jsel)
{
    LS_T0();
#ifdef PCG_DEV_ABL_SEL // dev ablation (wrong results, cost measurement only): no selection network
    val = cv[0];
    src = c.p < P ? c.p : 0u;
    jsel = 0;
    return;
#endif
    const uint32_t C = P * K;
    const bool act = c.p < P;
    const uint32_t R = C > np ? np + 1 : C;
    if constexpr (PCG_SEL_K32 && LP <= PCG_SEL_K32_LP) { // (LP = 32: 8 code bits leave near ties common, and the
                                              // 32-bit network beside the exact one spills: 1.12e6 ->
                                              // 6.7e5 cw/s on config 5, profiles/r04g_*)
        if (k32_select<LP, K>(c, cv, P, np, R, val, src, jsel)) {
            LS_STAMP(c, 50);
            return;
        }
    }
    uint64_t k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t code = (c.p << 3) | (uint32_t)j;
        const uint32_t o = (act && j < K) ? ord_of(cv[j]) : 0u;
        k[j] = ((uint64_t)o << 32) | (~code);
    }
#ifdef PCG_LS_FULL_LOCAL_SORT // dev: the general 19-comparator network
    local_sort<K>(k);
#else
    local_order<K>(k);
#endif
    float prev = 0.0f;
    bool tie = false;
    uint64_t mine = 0;
    if constexpr (PCG_SEL_VMERGE >= 2 || (PCG_SEL_VMERGE == 1 && LP <= 8)) {
        vmerge_select<LP, K>(c, k, P, np, R, val, src, jsel, tie);
    } else if constexpr (LP >= PCG_SEL_BITONIC_LP || K <= PCG_SEL_BITONIC_K) {
        bit_level<LP, K, 1>(k, c.p);
        mine = bit_pick<LP, K>(k, c.p, c.gb, np, R, tie);
    } else
    for (uint32_t r = 0; r < R; ++r) {
        uint64_t h = k[0];
        grp_kmax<LP>(h);
        const float bv = val_of((uint32_t)(h >> 32));
        tie = tie | ((r > 0) & (bv == prev));
        prev = bv;
        mine = (r < np && c.p == r) ? h : mine;
        const bool win = k[0] == h; // keys are unique: exactly one lane pops its head
#pragma unroll
        for (int j = 0; j < K - 1; ++j)
            k[j] = win ? k[j + 1] : k[j];
        k[K - 1] = win ? 0ull : k[K - 1];
    }
    if constexpr (!(PCG_SEL_VMERGE >= 2 || (PCG_SEL_VMERGE == 1 && LP <= 8))) {
        val = val_of((uint32_t)(mine >> 32));
        const uint32_t mc = ~(uint32_t)mine;
        src = (mc >> 3) & 31u;
        jsel = mc & 7u;
    }
    if (ballot(tie) == 0ull) {
        LS_STAMP(c, 50);
        return;
    }
    // literal simplePartialSortDescending per group (rare: exact metric ties)
    float* cval = c.gs + ls_gl_alpha_floats(c.mt, c.Sl) + c.gb * 8u;
    uint32_t* cid = reinterpret_cast<uint32_t*>(cval + 512);
    if (act) {
#pragma unroll
        for (uint32_t j = 0; j < K; ++j) {
            cval[c.p * K + j] = cv[j];
            cid[c.p * K + j] = c.p * K + j;
        }
    }
    wsync();
    if (c.p == 0) {
        const uint32_t lim = (C - 1) < np ? (C - 1) : np;
        for (uint32_t i = 0; i < lim; ++i) {
            uint32_t b = i;
            for (uint32_t j = i + 1; j < C; ++j)
                if (cval[j] > cval[b])
                    b = j;
            const float tv = cval[i];
            const uint32_t ti = cid[i];
            cval[i] = cval[b];
            cid[i] = cid[b];
            cval[b] = tv;
            cid[b] = ti;
        }
    }
    wsync();
    if (c.p < np) {
        val = cval[c.p];
        const uint32_t e = cid[c.p];
        src = e / K;
        jsel = e % K;
    }
    wsync();
}

// This lane takes the state of path `srcp`: its slot tables -- the LLR stages (and D
// bits) live on where they are (DataPool's lazy copy) -- and, with codeword rows, the row
// words [0, nw) decoded so far.  Converged code (bpermute); act = this lane survives.
template <int LP>
PCG_DEV void ls_dup(Ls<LP>& c, uint32_t srcp, uint32_t nw, bool act)
{
    LS_T0();
    const int sl = (int)(c.gb | srcp);
    const uint32_t lo = shfl((uint32_t)c.ptr, sl), hi = shfl((uint32_t)(c.ptr >> 32), sl);
    c.ptr = ((uint64_t)hi << 32) | lo;
    if constexpr (Ls<LP>::DB) {
        const uint32_t blo = shfl((uint32_t)c.bptr, sl), bhi = shfl((uint32_t)(c.bptr >> 32), sl);
        c.bptr = ((uint64_t)bhi << 32) | blo;
    } else {
        const lds_u32* srow = c.row_of((uint32_t)sl);
        lds_u32* row = c.row();
        // one wave's LDS instructions execute in order: every lane's read of a word
        // completes before any lane's write of it; 8 reads are issued before their writes
        uint32_t w = 0;
        for (; w + 8 <= nw; w += 8) {
            uint32_t x[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                x[u] = srow[(w + u) << 6];
            if (act) {
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    row[(w + u) << 6] = x[u];
            }
        }
        for (; w < nw; ++w) {
            const uint32_t x = srow[w << 6];
            if (act)
                row[w << 6] = x;
        }
    }
    LS_STAMP(c, 51);
}

// ---- branching leaves at n >= 8 (Rate-1 :353-413, SPC :498-621) ----------------------
template <int LP, typename Src>
PCG_DEV void ls_branch_leaf(Ls<LP>& c, Src src, uint32_t code, uint32_t s, uint32_t o, uint32_t& P)
{
    const uint32_t n = 1u << s;
    const uint32_t sl = s == c.top ? 0u : c.src_lane(s);
    const uint32_t kk = code == OP_S_R1 ? 2u : 4u;
    float T[4];
    uint32_t I[4], par = 0;
    LS_T0();
    if (n == 8) {
        const float4 a = src.ld(0, sl), b = src.ld(1, sl);
        const float v[8] = { a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w };
        weak8(v, kk, T, I, par);
    } else {
#ifdef PCG_DEV_ABL_WEAK // dev ablation (wrong results, cost measurement only): no weak-LLR search
        const float4 a = src.ld(0, sl);
        T[0] = fabs_(a.x); T[1] = fabs_(a.y); T[2] = fabs_(a.z); T[3] = fabs_(a.w);
        I[0] = 0; I[1] = 1; I[2] = 2; I[3] = 3;
        par = fbits(a.x);
#else
        bool done = false;
        if constexpr (PCG_WEAK_K32 && LP <= PCG_WEAK_K32_LP) // (config 5: +4 %, r04j_scl32_weak_k32_ab)
            done = kk == 2u ? weak_keys<LP, 3>(src, sl, n, kk, T, I, par) : weak_keys<LP, 5>(src, sl, n, kk, T, I, par);
        if (!done) {
            bool tie;
            weak_fast<LP>(src, sl, n, kk, T, I, par, tie);
            if (tie)
                ls_weak(c, src, sl, n, kk, T, I, par);
        }
#endif
    }
    LS_STAMP(c, 53);
    float cv[8];
    r1_spc_cands(code, c.m, T, par, cv);
    float val;
    uint32_t sp, j;
    uint32_t np;
    if (code == OP_S_R1) {
        const uint32_t C = P * 4;
        np = C < c.L ? C : c.L;
        ls_select<LP, 4>(c, cv, P, np, val, sp, j);
    } else {
        const uint32_t C = P * 8;
        np = C < c.L ? C : c.L;
        ls_select<LP, 8>(c, cv, P, np, val, sp, j);
    }
    const bool surv = c.p < np;
    // survivors take the source path's weak indices / parity and state
    const int sln = (int)(c.gb | sp);
    uint32_t Is[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
        Is[t] = shfl(I[t], sln);
    const uint32_t pars = shfl(par, sln);
    ls_dup(c, sp, (o + 31u) >> 5, surv);
    P = np;
    if (!surv)
        return;
    c.m = val;
    const uint32_t fm = ls_flip_sel(code, j, pars & 0x80000000u ? 1u : 0u);
    // hard decisions of the source path's leaf LLRs (its slot via the copied table)
    const uint32_t sl2 = s == c.top ? 0u : c.src_lane(s);
    for (uint32_t w0 = 0; w0 < n; w0 += 32) {
        const uint32_t nb = n < 32 ? n : 32u;
        uint32_t word = 0;
        constexpr int UB = 2 * Pre<Src>::U; // chunks loaded together
        float4 xq[UB];
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            if (q % UB == 0)
                ld_batch<UB>(src, (w0 >> 2) + q, (w0 + nb) >> 2, sl2, xq);
            if (q < nb / 4) {
                const float4 x = xq[q % UB];
                word |= ((fbits(x.x) >> 31) | ((fbits(x.y) >> 31) << 1) | ((fbits(x.z) >> 31) << 2) |
                         ((fbits(x.w) >> 31) << 3))
                        << (4u * q);
            }
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (((fm >> t) & 1u) && Is[t] >= w0 && Is[t] < w0 + nb)
                word ^= 1u << (Is[t] - w0);
        if constexpr (Ls<LP>::DB) {
            d_word(c, s, o, w0 >> 5, word);
        } else {
            lds_u32* row = c.row();
            const uint32_t pos = o + w0;
            if (nb == 32) {
                row[(pos >> 5) << 6] = word;
            } else {
                const uint32_t sh = pos & 31u, msk = ((1u << nb) - 1u) << sh;
                lds_u32* wp = row + ((pos >> 5) << 6);
                *wp = (*wp & ~msk) | (word << sh);
            }
        }
    }
    if constexpr (Ls<LP>::DB)
        d_end(c, s, o);
}

// ---- size-8 subtrees in registers (ShortRateRNode(8), scl_avx_float.cpp:273-307) -----
struct LsSt8 {
    float x8[8];
    float a4[4];
    uint32_t bits; // bit i = codeword position o + i
    uint32_t root; // path index at subtree entry
    uint32_t P;
    bool branched;
};

PCG_DEV float ordered8(const float (&a)[8])
{
    return a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6] + a[7];
}

// candidates of a leaf of size n (2 or 4) on v[0..n): cv[0..k) and per-candidate n-bit
// patterns packed 4 bits each into pat (REP :428-481, R1 :365-379, SPC :511-585).
PCG_DEV void st_cands8(uint32_t kind, const float (&v)[4], uint32_t n, float m, float (&cv)[8], uint32_t& pat)
{
    const uint32_t nmask = (1u << n) - 1u;
#pragma unroll
    for (int j = 0; j < 8; ++j)
        cv[j] = 0.0f;
    if (kind == ST_REP) { // zero padded to 8 lanes
        float z[8], o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float l = j < (int)n && j < 4 ? v[j & 3] : 0.0f;
            z[j] = 0.0f + minps(l, 0.0f);
            o[j] = 0.0f + maxps(l, 0.0f);
        }
        cv[0] = m + ordered8(z);
        cv[1] = m - ordered8(o);
        pat = nmask << 4;
        return;
    }
    float T[4];
    uint32_t I[4], base = 0, par = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        T[j] = fabs_(v[j]);
        I[j] = (uint32_t)j;
        if (j < (int)n) {
            par ^= fbits(v[j]);
            base |= (fbits(v[j]) >> 31) << j;
        }
    }
    const uint32_t kk = kind == ST_R1 ? 2u : 4u;
    const uint32_t lim = (n - 1) < kk ? (n - 1) : kk;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        if (t < (int)lim) {
            float bv = T[t];
            uint32_t b = (uint32_t)t;
#pragma unroll
            for (int j = t + 1; j < 4; ++j) {
                const bool better = j < (int)n && T[j] < bv;
                bv = better ? T[j] : bv;
                b = better ? (uint32_t)j : b;
            }
            const uint32_t tv = fbits(T[t]), ti = I[t];
            uint32_t bi = I[t];
#pragma unroll
            for (int j = t + 1; j < 4; ++j) {
                const uint32_t mj = 0u - (uint32_t)(b == (uint32_t)j);
                bi = (I[j] & mj) | (bi & ~mj);
                T[j] = ubits((tv & mj) | (fbits(T[j]) & ~mj));
                I[j] = (ti & mj) | (I[j] & ~mj);
            }
            T[t] = bv;
            I[t] = bi;
        }
    }
    const uint32_t ib[4] = { 1u << I[0], 1u << I[1], 1u << I[2], 1u << I[3] };
    if (kind == ST_R1) {
        cv[0] = m;
        cv[1] = m - T[0];
        cv[2] = m - T[1];
        cv[3] = m - T[0] - T[1];
        pat = base | ((base ^ ib[0]) << 4) | ((base ^ ib[1]) << 8) | ((base ^ ib[0] ^ ib[1]) << 12);
        return;
    }
    const bool odd = (par & 0x80000000u) != 0;
    float mm = m, pinv = 1.0f;
    if (odd) {
        pinv = 0.0f;
        mm -= T[0];
    }
    cv[0] = mm;
    cv[1] = mm - pinv * T[0] - T[1];
    cv[2] = mm - pinv * T[0] - T[2];
    cv[3] = mm - pinv * T[0] - T[3];
    cv[4] = mm - T[1] - T[2];
    cv[5] = mm - T[1] - T[3];
    cv[6] = mm - T[2] - T[3];
    cv[7] = mm - pinv * T[0] - T[1] - T[2] - T[3];
    pat = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t fm = ls_flip_sel(OP_S_SPC, j, odd ? 1u : 0u);
        uint32_t fl = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            fl |= ((fm >> q) & 1u) ? ib[q] : 0u;
        pat |= ((base ^ fl) & nmask) << (4 * j);
    }
}

template <int LP>
PCG_DEV void st8_r0(Ls<LP>& c, const float (&v)[4], uint32_t n)
{
    float q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        q[j] = 0.0f + minps(j < (int)n && j < 4 ? v[j & 3] : 0.0f, 0.0f);
    c.m = c.m + ordered8(q);
}

template <int LP>
PCG_DEV void st8_branch(Ls<LP>& c, LsSt8& st, uint32_t kind, const float (&v)[4], uint32_t n, uint32_t boff)
{
    float cv[8];
    uint32_t pat = 0;
    st_cands8(kind, v, n, c.m, cv, pat);
    float val;
    uint32_t sp, j, np;
    if (kind == ST_R1) {
        const uint32_t C = st.P * 4;
        np = C < c.L ? C : c.L;
        ls_select<LP, 4>(c, cv, st.P, np, val, sp, j);
    } else if (kind == ST_SPC) {
        const uint32_t C = st.P * 8;
        np = C < c.L ? C : c.L;
        ls_select<LP, 8>(c, cv, st.P, np, val, sp, j);
    } else {
        const uint32_t C = st.P * 2;
        np = C < c.L ? C : c.L;
        ls_select<LP, 2>(c, cv, st.P, np, val, sp, j);
    }
    LS_T0();
    const int sl = (int)(c.gb | sp);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        st.x8[i] = shfl(st.x8[i], sl);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        st.a4[i] = shfl(st.a4[i], sl);
    st.bits = shfl(st.bits, sl);
    st.root = shfl(st.root, sl);
    pat = shfl(pat, sl);
    st.bits |= ((pat >> (4 * j)) & ((1u << n) - 1u)) << boff;
    c.m = val;
    st.P = np;
    st.branched = true;
    LS_STAMP(c, 52);
}

template <int LP>
PCG_DEV void st8_child2(Ls<LP>& c, LsSt8& st, uint32_t kind, const float (&a2)[4], uint32_t boff)
{
    if (kind == ST_R0)
        st8_r0(c, a2, 2);
    else
        st8_branch(c, st, kind, a2, 2, boff);
}

template <int LP>
PCG_DEV void st8_child4(Ls<LP>& c, LsSt8& st, uint32_t d, uint32_t boff)
{
    const uint32_t kind = d & 7u;
    if (kind == ST_R0) {
        st8_r0(c, st.a4, 4);
    } else if (kind != ST_RATER) {
        const float v[4] = { st.a4[0], st.a4[1], st.a4[2], st.a4[3] };
        st8_branch(c, st, kind, v, 4, boff);
    } else { // ShortRateRNode(4): F, left(2), G, right(2), CombineBitsShort
        float a2[4] = { polar_f(st.a4[0], st.a4[2]), polar_f(st.a4[1], st.a4[3]), 0.0f, 0.0f };
        st8_child2(c, st, (d >> 3) & 3u, a2, boff);
        a2[0] = polar_g_bit(st.a4[0], st.a4[2], st.bits, boff);
        a2[1] = polar_g_bit(st.a4[1], st.a4[3], st.bits, boff + 1);
        st8_child2(c, st, (d >> 5) & 3u, a2, boff + 2);
        st.bits ^= ((st.bits >> (boff + 2)) & 3u) << boff;
    }
}

template <int LP, typename Src>
PCG_DEV void ls_st8(Ls<LP>& c, Src src, uint32_t desc, uint32_t o, uint32_t& P)
{
    LsSt8 st;
    st.P = P;
    st.branched = false;
    st.root = c.p;
    st.bits = 0;
    {
        const uint32_t sl = c.top == 3 ? 0u : c.src_lane(3);
        const float4 lo = src.ld(0, sl), hi = src.ld(1, sl);
        st.x8[0] = lo.x; st.x8[1] = lo.y; st.x8[2] = lo.z; st.x8[3] = lo.w;
        st.x8[4] = hi.x; st.x8[5] = hi.y; st.x8[6] = hi.z; st.x8[7] = hi.w;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
        st.a4[i] = polar_f(st.x8[i], st.x8[i + 4]);
    st8_child4(c, st, desc & 0xffu, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        st.a4[i] = polar_g_bit(st.x8[i], st.x8[i + 4], st.bits, (uint32_t)i);
    st8_child4(c, st, (desc >> 8) & 0xffu, 4);
    st.bits ^= (st.bits >> 4) & 0xFu; // CombineBitsShort(4)
    // the 8 bits into D[4] or the row; after branching, first take the state (slot tables,
    // row prefix) of the path each survivor descends from
    const uint32_t sh = o & 31u, wo = o >> 5, msk = 0xFFu << sh;
    if (st.branched)
        ls_dup(c, st.root, wo + 1, c.p < st.P);
    P = st.P;
    if (c.p < P) {
        if constexpr (Ls<LP>::DB) {
            d_word(c, 3, o, 0, st.bits);
            d_end(c, 3, o);
        } else {
            lds_u32* w = c.row() + (wo << 6);
            *w = (*w & ~msk) | (st.bits << sh);
        }
    }
}

// ---- CRC check of a path's codeword (the plan's GF(2) syndrome model) -----------------
// The syndrome of the info bits is affine in them (plan.cpp); in codeword coordinates
// bit r of it is c0_r ^ parity(sum_w popcount(word_w & rows[r][w])): W * CB and +
// popcount pairs per lane, the masks wave-uniform scalar loads.
template <int CB>
PCG_DEV uint32_t crc_syn(const DBits& cw, const uint32_t* rows, uint32_t W, uint32_t c0)
{
    uint32_t acc[CB];
#pragma unroll
    for (int r = 0; r < CB; ++r)
        acc[r] = 0;
#pragma unroll 4
    for (uint32_t w = 0; w < W; ++w) {
        const uint32_t word = cw.word(w);
#pragma unroll
        for (int r = 0; r < CB; ++r)
            acc[r] += (uint32_t)__builtin_popcount(word & ld_const(rows, r * W + w));
    }
    uint32_t syn = c0;
#pragma unroll
    for (int r = 0; r < CB; ++r)
        syn ^= (acc[r] & 1u) << r;
    return syn;
}

// ---- punctured frames ------------------------------------------------------------------
// Scratch floats of one wave without the channel region (alpha slab, tie list, D region);
// punctured launches append the wave's G depunctured frames (G x N floats) after them.
constexpr __host__ __device__ inline uint64_t ls_scratch_floats(uint32_t top, uint32_t mt, uint32_t Sl, uint32_t Sb)
{
    return ls_gl_alpha_floats(mt, Sl) + 1024ull + 64ull * ls_dgl_words(top, Sb);
}
// pcg_decode_punctured_f32 on a list plan: the wave's G received frames (E LLRs each) are
// depunctured into its scratch slab -- position j = llr[pmap[j]] or +0.0 (puncturer.h:92-99:
// fill with zeros, then scatter, here as a gather over the output) -- and every channel read of
// the walk (c.y, the staged root-child DMA included) uses that copy: no separate depuncture pass
// and no F x N staging buffer in HBM.  (Invalid slots of a partial group copy the last frame.)
template <int LP>
PCG_DEV void ls_depuncture(Ls<LP>& c, const KernelArgs& a, uint64_t frame)
{
    constexpr uint32_t G = 64 / LP;
    float* ch = c.gs + ls_scratch_floats(c.top, c.mt, c.Sl, c.Sb);
    const uint32_t q = c.N >> 2; // float4 per frame
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t lo = shfl((uint32_t)frame, (int)(g * LP)), hi = shfl((uint32_t)(frame >> 32), (int)(g * LP));
        const float* row = a.llr + ((((uint64_t)hi << 32) | lo) * a.in_stride);
#pragma unroll 2
        for (uint32_t t = c.lane; t < q; t += 64) {
            const int4 s = *reinterpret_cast<const int4*>(a.pmap + 4u * t);
            float4 v;
            v.x = s.x >= 0 ? row[s.x] : 0.0f;
            v.y = s.y >= 0 ? row[s.y] : 0.0f;
            v.z = s.z >= 0 ? row[s.z] : 0.0f;
            v.w = s.w >= 0 ? row[s.w] : 0.0f;
            *reinterpret_cast<float4*>(ch + g * c.N + 4u * t) = v;
        }
    }
    wsync();
    c.y = ch + (c.lane / LP) * c.N;
}

// ---- the kernel ------------------------------------------------------------------------
#ifndef PCG_LS_MINW
#define PCG_LS_MINW 2
#endif
// One op of the walk, then a wave barrier.  fuse: this F / G runs fused with the next
// schedule op, the child's F (ls_fgf); desc: a size-8 subtree's descriptor word.
template <int LP>
PCG_DEV void ls_op(Ls<LP>& c, uint32_t code, uint32_t s, uint32_t o, uint32_t& P, bool fuse, uint32_t desc)
{
    const bool act = c.p < P;
    switch (code) {
    case OP_F:
        if (fuse)
            ls_fgf_op<OP_F>(c, s, o, P);
        else
            ls_fg_op<OP_F>(c, s, o, P);
        break;
    case OP_G:
        if (fuse)
            ls_fgf_op<OP_G>(c, s, o, P);
        else
            ls_fg_op<OP_G>(c, s, o, P);
        break;
    case OP_COMB:
        ls_comb(c, s, o, act);
        break;
    case OP_S_ST8:
        with_stage(c, 3, o, [&](auto src) { ls_st8(c, src, desc, o, P); });
        break;
    case OP_S_R0:
        with_stage(c, s, o, [&](auto src) { ls_r0(c, src, s, o, act); });
        break;
    default: // OP_S_R1 / OP_S_SPC (n >= 8)
        with_stage(c, s, o, [&](auto src) { ls_branch_leaf(c, src, code, s, o, P); });
        break;
    }
    wsync();
}

#ifdef PCG_RTC
// Plan-specialised walk (rtc.cpp): the plan's schedule as literals (PCG_RTC_OPS), unrolled
// at compile time with every op's code, stage, offset, fusion and descriptor constant
// (PCG_RTC_UNROLL = 1; measured: config 3's kernel did not compile within 20 minutes).  By
// default the specialised list kernel keeps the schedule loop and only its layout and plan
// constants are literals (scl_rtc_kernel).
constexpr uint32_t rtc_ops[] = { PCG_RTC_OPS };
constexpr uint32_t rtc_nops = sizeof(rtc_ops) / sizeof(rtc_ops[0]);
constexpr uint32_t rtc_mt = ls_mtop(PCG_RTC_LOG2N, PCG_RTC_VIRT);

template <int LP, uint32_t K>
PCG_DEV void ls_walk(Ls<LP>& c, uint32_t& P)
{
    if constexpr (K < rtc_nops) {
        constexpr uint32_t w = rtc_ops[K];
        constexpr uint32_t code = op_code(w), s = op_stage(w), o = op_off(w);
        constexpr bool fuse = (code == OP_F || code == OP_G) && s >= 5 && s - 1 >= PCG_RTC_SL && s - 1 < rtc_mt &&
                              (PCG_RTC_FUSE & 1u) && K + 1 < rtc_nops && op_code(rtc_ops[K + 1]) == OP_F &&
                              op_stage(rtc_ops[K + 1]) == s - 1;
        constexpr bool d = code == OP_S_ST8;
        constexpr uint32_t desc = d ? rtc_ops[K + 1] : 0u;
        ls_op<LP>(c, code, s, o, P, fuse, desc);
        ls_walk<LP, K + (fuse || d ? 2u : 1u)>(c, P);
    }
}
#endif

template <int LP>
PCG_DEV void sclls_body(const KernelArgs& a)
{
    extern __shared__ float smem[];
    constexpr uint32_t G = 64 / LP;
    Ls<LP> c;
    c.lds = smem;
#ifdef PCG_LS_PROF
    uint64_t* lprof = reinterpret_cast<uint64_t*>(smem + a.wave_lds_floats);
    c.lprof = lprof;
    if (threadIdx.x == 0)
        for (int b = 0; b < 192; ++b) // cycles, then requested read / write bytes per bucket
            lprof[b] = 0;
    wsync();
#endif
    c.N = a.N;
    c.L = a.L;
    c.top = a.log2N;
    c.Sl = a.lds_stage_limit;
    c.mt = ls_mtop(c.top, a.scl_virt);
    c.vlow = a.scl_v3;
    c.ab = ls_abase(c.vlow);
    c.Sb = a.scl_sb;
    c.ly = ls_layout(c.top, a.lds_stage_limit, c.vlow, c.Sb);
    c.lane = threadIdx.x;
    c.share = (a.scl_fuse >> 1) & 1u;
    c.stage_root = (a.scl_fuse >> 2) & 1u;
    c.p = c.lane & (LP - 1);
    c.gb = c.lane & ~(uint32_t)(LP - 1);
    c.gs = a.scratch + (uint64_t)blockIdx.x * a.scratch_floats;
    c.dl = (lds_u32*)(smem + c.ly.d);
    c.dg = (gl_u32*)(c.gs + ls_gl_alpha_floats(c.mt, c.Sl) + 1024u); // after the tie region
    const uint32_t W = a.N >= 32 ? a.N / 32 : 1u;

    const uint64_t Fn = a.fcount ? (uint64_t)*a.fcount : a.F;
#if PCG_LS_STAGGER > 0
    // Start stagger: every wave would otherwise run the first codeword group's ops in step with
    // all the others (the same staged channel rounds, the same slab stages at the same time), and
    // the first round of a launch then takes ~1.6x a steady-state round.  A pseudo-random delay
    // of 0..15 steps of ~3.4 us desynchronises them (launches of >= 2 groups per wave only: a
    // one-round launch, e.g. an adaptive plan's list stage, would just wait).
    if (Fn >= 2ull * G * gridDim.x) {
        const uint32_t steps = ((blockIdx.x * 2654435761u) >> 28) * (uint32_t)PCG_LS_STAGGER;
        for (uint32_t i = 0; i < steps; ++i)
            __builtin_amdgcn_s_sleep(127);
    }
#endif
    // codeword groups: from the plan's work queue (dynamic balance across SIMDs whose
    // resident wave counts differ), else a static grid stride
    const uint64_t stride = (uint64_t)gridDim.x * G;
    for (uint64_t fb = a.queue ? queue_next(a.queue) * G : (uint64_t)blockIdx.x * G; fb < Fn;
         fb = a.queue ? queue_next(a.queue) * G : fb + stride) {
        const uint64_t slot = fb + c.lane / LP;
        const bool fvalid = slot < Fn;
        const uint64_t fs = fvalid ? slot : Fn - 1;
        const uint64_t frame = a.fmap ? (uint64_t)a.fmap[fs] : fs;
        c.y = a.llr + frame * a.N;
        if (a.pmap) // punctured frames: depunctured into the wave's scratch first
            ls_depuncture<LP>(c, a, frame);
        // path 0 starts at 0 (a freshly constructed decoder) or, for a reused decoder
        // instance, at the previous frame's final path-0 metric
        c.m = a.metric0;
        c.ptr = 0;
        c.bptr = 0;
        c.fin = false;
        uint32_t P = 1;
#ifdef PCG_LS_PROF
        const uint64_t tf0 = __builtin_amdgcn_s_memtime();
#endif
#if defined(PCG_RTC) && PCG_RTC_UNROLL
        ls_walk<LP, 0>(c, P);
#else
        for (uint32_t kop = 0; kop < a.nops; ++kop) {
#ifdef PCG_LS_PROF
            const uint32_t kop0 = kop;
#endif
            const uint32_t w = ld_const(a.ops, kop);
            const uint32_t code = op_code(w), s = op_stage(w), o = op_off(w);
#ifdef PCG_LS_PROF
            const uint64_t t0 = __builtin_amdgcn_s_memtime();
            if (c.lane == 0) {
                ls_gb_ctr()[0] = 0;
                ls_gb_ctr()[1] = 0;
            }
#endif
            // an F/G whose output stage is in the global slab and whose next op is the
            // child's F runs fused with it (ls_fgf)
            bool fuse = false;
            if ((code == OP_F || code == OP_G) && s >= 5 && s - 1 >= c.Sl && s - 1 < c.mt && (a.scl_fuse & 1u) &&
                kop + 1 < a.nops) {
                const uint32_t w2 = ld_const(a.ops, kop + 1);
                fuse = op_code(w2) == OP_F && op_stage(w2) == s - 1;
            }
            const uint32_t desc = code == OP_S_ST8 ? ld_const(a.ops, kop + 1) : 0u;
            ls_op<LP>(c, code, s, o, P, fuse, desc);
            if (fuse || code == OP_S_ST8)
                ++kop; // the fused child F / the subtree's descriptor word
#ifdef PCG_LS_PROF
            {
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                uint32_t b = code;
                if (code == OP_F || code == OP_G)
                    b += s >= c.mt ? 16u : s >= c.Sl ? 8u : (s - 1 >= c.Sl ? 24u : 0u);
                if (c.lane == 0) {
                    lprof[b] += t1 - t0;
                    lprof[64 + b] += ls_gb_ctr()[0];
                    lprof[128 + b] += ls_gb_ctr()[1];
#ifdef PCG_LS_PROF_POS // dev: the cycles of every schedule position (tools/ls_prof_pos.py)
                    if (a.prof && kop0 < 3840u)
                        atomicAdd(&a.prof[256u + kop0], (unsigned long long)(t1 - t0));
#endif
                }
            }
#endif
        }
#endif
#ifdef PCG_LS_PROF
        const uint64_t tf1 = __builtin_amdgcn_s_memtime();
#endif
        // extractBestPath (scl_avx_float.cpp:711-750): first path in list order whose
        // detector check passes, else path 0.
        // (every active path's codeword is in its own lane: the root's op wrote it, to D[top]
        // or, fin, to the LDS stage region)
        const bool act = c.p < P;
        const uint32_t top = c.top;
        const lds_u32* fr = (const lds_u32*)(c.lds + c.ly.alpha);
        auto cw_of = [&](uint32_t l) {
            if constexpr (!Ls<LP>::DB)
                return rowbits(c, l, 0u);
            return c.fin ? DBits{ fr, nullptr, l, false, 0u } : dbits(c, top, l);
        };
        if (!a.systematic && act) {
            lds_u32* f = Ls<LP>::DB ? (lds_u32*)(c.lds + c.ly.alpha) + c.lane : c.row();
            const bool lf = !Ls<LP>::DB || c.fin;
            auto ld = [&](uint32_t wi) { return lf ? f[wi << 6] : c.dld(top, wi, c.lane); };
            auto st = [&](uint32_t wi, uint32_t v) {
                if (lf)
                    f[wi << 6] = v;
                else
                    c.dst(top, wi, v);
            };
            for (uint32_t wi = 0; wi < W; ++wi)
                st(wi, transform_word(ld(wi), a.N));
            for (uint32_t d = 1; d < W; d <<= 1)
                for (uint32_t wi = 0; wi < W; ++wi)
                    if (!(wi & d))
                        st(wi, ld(wi) ^ ld(wi + d));
        }
        wsync();
        // detector syndrome: bit r = c0_r ^ parity(codeword & row mask r)
        const DBits cw = cw_of(c.lane);
        uint32_t syn;
        switch (a.crc_bits) {
        case 8: syn = crc_syn<8>(cw, a.crc_rows, W, a.crc_c0); break;
        case 11: syn = crc_syn<11>(cw, a.crc_rows, W, a.crc_c0); break;
        case 16: syn = crc_syn<16>(cw, a.crc_rows, W, a.crc_c0); break;
        case 32: syn = crc_syn<32>(cw, a.crc_rows, W, a.crc_c0); break;
        default: syn = a.crc_c0; break;
        }
        const uint64_t okm = ballot(act && syn == 0u);
        const uint32_t gm = (uint32_t)((okm >> c.gb) & (LP == 64 ? ~0ull : ((1ull << LP) - 1ull)));
        const uint32_t chosen = gm ? (uint32_t)__builtin_ctz(gm) : 0u;
        const DBits crow = cw_of(c.gb | chosen);
        if (fvalid) {
            for (uint32_t b = c.p; b < a.kb; b += LP) {
                uint32_t byte = 0;
                for (uint32_t j = 0; j < 8; ++j) {
                    const uint32_t idx = 8 * b + j;
                    if (idx < a.K) {
                        const uint32_t ps = a.info_pos[idx];
                        byte |= (crow.at(ps) & 1u) << (7 - j);
                    }
                }
                a.info[frame * a.kb + b] = (uint8_t)byte;
            }
            if (c.p == 0 && a.ok)
                a.ok[frame] = gm ? 1 : 0;
            if (a.metrics && c.p < a.L)
                a.metrics[frame * a.L + c.p] = act ? c.m : 0.0f;
        }
        wsync();
#ifdef PCG_LS_PROF
        if (c.lane == 0) {
            const uint64_t tf2 = __builtin_amdgcn_s_memtime();
            lprof[60] += tf2 - tf1; // extractBestPath + output
            lprof[61] += tf2 - tf0; // whole codeword group
            lprof[62] += 1;
        }
#endif
    }
#ifdef PCG_LS_PROF
    wsync();
    if (c.lane == 0 && a.prof)
        for (int b = 0; b < 192; ++b)
            if (lprof[b])
                atomicAdd(&a.prof[b], (unsigned long long)lprof[b]);
#endif
}

// Translation units (not hiprtc): the host part -- layout, occupancy, dispatch -- is the object
// built without PCG_LS_INST; each list width's kernel is its own object (Makefile:
// -DPCG_LS_INST=<LP>), so the five instantiations compile in parallel.  A dev build
// (tools/build_dev_lib.sh) compiles one width together with the host part (-DPCG_LS_HOST).
#ifndef PCG_RTC
#ifndef PCG_LS_INST
#define PCG_LS_INST 0
#endif
#if PCG_LS_INST == 0 && !defined(PCG_LS_HOST)
#define PCG_LS_HOST 1
#endif
#if PCG_LS_INST
template <int LP>
__global__ void __launch_bounds__(64, PCG_LS_MINW) sclls_kernel(KernelArgs a)
{
    sclls_body<LP>(a);
}
#endif
#endif

} // namespace

#ifdef PCG_RTC
// the plan-specialised list decoder: the layout and the plan's constants are literals
extern "C" __global__ void __launch_bounds__(64, PCG_LS_MINW) scl_rtc_kernel(KernelArgs a)
{
    KernelArgs b = a;
    b.N = PCG_RTC_N;
    b.log2N = PCG_RTC_LOG2N;
    b.K = PCG_RTC_K;
    b.kb = (PCG_RTC_K + 7u) / 8u;
    b.L = PCG_RTC_L;
    b.crc_bits = PCG_RTC_CRC;
    b.systematic = PCG_RTC_SYS;
    b.lds_stage_limit = PCG_RTC_SL;
    b.scl_virt = PCG_RTC_VIRT;
    b.scl_v3 = PCG_RTC_V3;
    b.scl_sb = PCG_RTC_SB;
    b.scl_fuse = PCG_RTC_FUSE;
    b.scl_lp = PCG_RTC_LP;
    b.nops = rtc_nops;
    sclls_body<PCG_RTC_LP>(b);
}
#else // host side: layout, occupancy, launch

#define PCG_LS_CAT2(x, y) x##y
#define PCG_LS_CAT(x, y) PCG_LS_CAT2(x, y)
// per-width entry points of the kernel objects: resident waves per CU at an LDS size, launch
#define PCG_LS_DECL(W)                                                                                    \
    int PCG_LS_CAT(sclls_resident_, W)(uint32_t lds_bytes);                                               \
    int PCG_LS_CAT(sclls_launch_, W)(const KernelArgs& a, size_t lds, hipStream_t stream);
PCG_LS_DECL(2)
PCG_LS_DECL(4)
PCG_LS_DECL(8)
PCG_LS_DECL(16)
PCG_LS_DECL(32)

#if PCG_LS_INST
int PCG_LS_CAT(sclls_resident_, PCG_LS_INST)(uint32_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, sclls_kernel<PCG_LS_INST>, 64, lds_bytes) != hipSuccess)
        n = 0;
    return n;
}
int PCG_LS_CAT(sclls_launch_, PCG_LS_INST)(const KernelArgs& a, size_t lds, hipStream_t stream)
{
    hipLaunchKernelGGL(sclls_kernel<PCG_LS_INST>, dim3(a.units), dim3(64), lds, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
#endif

#ifdef PCG_LS_HOST
#ifndef PCG_SCL_VIRT_DEFAULT
#define PCG_SCL_VIRT_DEFAULT 3 // recomputed top stages (2: the quarters too, 3: eighths for LP >= 16, where sclls_layout allows)
#endif
int sclls_layout(uint32_t N, uint32_t L, uint32_t lp, uint32_t vleaf, uint32_t* wave_lds_floats,
                 uint32_t* lds_stage_limit, uint64_t* scratch_floats, uint32_t* virt, uint32_t* v3, uint32_t* sb)
{
    const bool db = lp >= PCG_LS_DBITS_LP;
    if (L < 2 || L > 32 || N < 8)
        return -4;
#if PCG_LS_INST
    // a development build (tools/build_dev_lib.sh) rebuilt one list width with its knobs: plans of
    // the other widths are refused at creation (PCG_E_UNSUPPORTED), not only at launch
    if (lp != PCG_LS_INST)
        return -4;
#endif
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    if (top > 3 + 12) // 5-bit slot fields for stages 3 .. top-1 in 64 bits
        return -4;
    // stage 3 recomputed from stored stage-4 chunks (N >= 64); PCG_SCL_V3 = 0 stores it,
    // 2 also recomputes stage 4 from stage 5 (N >= 128)
    uint32_t w3 = top >= 6 ? 1u : 0u;
    if (const char* e = getenv("PCG_SCL_V3")) {
        const uint32_t v = (uint32_t)atoi(e);
        w3 = v == 0 ? 0u : (v >= 2 && top >= 7 ? 2u : w3);
    }
    // floats per wave.  Rows: 24 KB (N = 1024, L = 8: S_l = 6, stages 4-5 and the rows in
    // LDS: 20 KB, 8 waves/CU); D buffers: 20 KB = 8 waves/CU, the VGPR limit too (N = 4096:
    // LLR stages 4-5 and D stages 4-9)
    uint32_t budget = (db ? 20 : 24) * 1024 / 4;
    const uint32_t bitsf = 64u * (N >= 32 ? N / 32 : 1u);
    if (!db && bitsf + 2048u > budget) // large N: the rows alone fill 24 KB; keep stages 3-4 on chip
        budget = bitsf + 2048u;
    if (const char* e = getenv("PCG_SCL_LDS_KB"))
        budget = (uint32_t)atoi(e) * 1024 / 4;
    // virt = V >= 2 (stages top-1 .. top-V recomputed, the deepest inside its staged F/G ops,
    // ls_fgf_rootv) needs: no leaf at stage >= top-V with both fusions on (the caller's vleaf
    // >= V), V = 3 only for LP >= 16, stage top-V >= 7 (8-chunk bit words), the recomputed
    // nodes' grandchildren in the slab and the LDS stage region holding one staging round
    // (checked below, else one level less)
    uint32_t vmax = ls_max_virt(top);
    if (lp >= 16 && top >= 10 && vleaf >= 3)
        vmax = 3;
    while (vmax >= 2 && (vleaf < vmax || top < 7 + vmax))
        --vmax;
    uint32_t vt = vmax < PCG_SCL_VIRT_DEFAULT ? vmax : PCG_SCL_VIRT_DEFAULT;
    if (const char* e = getenv("PCG_SCL_VIRT")) {
        const uint32_t v = (uint32_t)atoi(e);
        vt = v < vmax ? v : vmax;
    }
    auto stage_limit = [&](uint32_t mtv, uint32_t Sbv) {
        uint32_t S = mtv;
        while (S > LS_MINS && ls_layout(top, S, w3, Sbv).total > budget)
            --S;
        return S;
    };
    while (vt >= 2) {
        uint32_t Sb0 = top + 1 < 8u ? top + 1 : 8u;
        Sb0 = !db ? 0u : (Sb0 < 5u ? 5u : Sb0);
        const uint32_t S = stage_limit(ls_mtop(top, vt), Sb0), ab = ls_abase(w3);
        const uint32_t region = (1u << S) > ab ? 4u * 64u * ((1u << S) - ab) : 0u;
        const uint32_t kc = 4u << vt; // staged channel chunks per output chunk (fused)
        const uint32_t mneed = lp / kc > 1u ? lp / kc : 1u;
        if (S + vt + 2u <= top && (64u / lp) * kc * mneed * 16u <= region)
            break;
        --vt;
    }
    const uint32_t mt = ls_mtop(top, vt);
    // LDS: the small D stages (4-7: every leaf and Combine writes one), then LLR stages up
    // from 3+v3, then the larger D stages while they fit
    uint32_t Sb = top + 1 < 8u ? top + 1 : 8u;
    Sb = !db ? 0u : (Sb < 5u ? 5u : Sb);
    uint32_t Sl = stage_limit(mt, Sb);
    if (const char* e = getenv("PCG_SCL_STAGE_LIMIT"); e && vt < 2) {
        const uint32_t v = (uint32_t)atoi(e);
        if (v >= LS_MINS && v <= mt)
            Sl = v;
    }
    while (db && Sb <= top && ls_layout(top, Sl, w3, Sb + 1).total <= budget)
        ++Sb;
    if (const char* e = getenv("PCG_SCL_SB"); e && db) {
        const uint32_t v = (uint32_t)atoi(e);
        if (v >= 5 && v <= top + 1)
            Sb = v;
    }
    const LsLayout ly = ls_layout(top, Sl, w3, Sb);
    if (ly.total * 4 > 160 * 1024)
        return -4;
    *wave_lds_floats = ly.total;
    *lds_stage_limit = Sl;
    *scratch_floats = ls_scratch_floats(top, mt, Sl, Sb);
    *virt = vt;
    *v3 = w3;
    *sb = Sb;
    return 0;
}

std::string sclls_rtc_defines(bool* nondefault)
{
    // (the knobs' values in this translation unit: a dev build's -D flags reach the hiprtc
    // source too, so its specialised kernel is the variant's, with the layout computed here)
    std::string s;
    bool nd = false;
    auto d = [&](const char* k, long v, long dflt) {
        s += std::string("#define ") + k + " " + std::to_string(v) + "\n";
        nd = nd || v != dflt;
    };
    d("PCG_LS_DBITS_LP", PCG_LS_DBITS_LP, 16);
    d("PCG_FGF_U", PCG_FGF_U, 1);
    d("PCG_STG_GM", PCG_STG_GM, 1);
    d("PCG_STG_DB", PCG_STG_DB, 1);
    d("PCG_DEEP_SHARE", PCG_DEEP_SHARE, 1);
    d("PCG_F_OLD", PCG_F_OLD, 0);
    d("PCG_SEL_TOP8", PCG_SEL_TOP8, 1);
    d("PCG_STG_SHARED_F", PCG_STG_SHARED_F, 1);
    d("PCG_STG_RING", PCG_STG_RING, 2);
    d("PCG_STG_TAIL_DRAIN", PCG_STG_TAIL_DRAIN, 0);
    d("PCG_LS_STAGGER", PCG_LS_STAGGER, 2);
#ifdef PCG_DEV_ABL_DEEP
    d("PCG_DEV_ABL_DEEP", PCG_DEV_ABL_DEEP, 0);
#endif
    d("PCG_SEL_BITONIC_LP", PCG_SEL_BITONIC_LP, 16);
    d("PCG_SEL_BITONIC_K", PCG_SEL_BITONIC_K, 4);
    d("PCG_SEL_VMERGE", PCG_SEL_VMERGE, 0);
    d("PCG_SEL_K32", PCG_SEL_K32, 1);
    d("PCG_SEL_K32_LP", PCG_SEL_K32_LP, 8);
    d("PCG_WEAK_K32", PCG_WEAK_K32, 1);
    d("PCG_WEAK_K32_LP", PCG_WEAK_K32_LP, 32);
    d("PCG_LS_MINW", PCG_LS_MINW, 2);
#ifdef PCG_LS_FULL_LOCAL_SORT
    s += "#define PCG_LS_FULL_LOCAL_SORT 1\n";
    nd = true;
#endif
#ifdef PCG_LS_PROF
    s += "#define PCG_LS_PROF 1\n";
    nd = true;
#endif
    if (nondefault)
        *nondefault = nd;
    return s;
}

static uint32_t lp_of(uint32_t L)
{
    uint32_t lp = 2;
    while (lp < L)
        lp <<= 1;
    return lp;
}

// Waves (= scratch units) for a launch of F frames: one persistent wave per resident
// slot (hipOccupancy: VGPR / LDS limits), capped at PCG_SCL_WPC waves per CU.
uint64_t sclls_wave_cap(uint32_t lp, uint32_t wave_lds_floats)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess)
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint32_t lds = wave_lds_floats * 4u;
    int res = 0;
    switch (lp) {
    case 2: res = sclls_resident_2(lds); break;
    case 4: res = sclls_resident_4(lds); break;
    case 8: res = sclls_resident_8(lds); break;
    case 16: res = sclls_resident_16(lds); break;
    default: res = sclls_resident_32(lds); break;
    }
    uint64_t wpc = res > 0 ? (uint64_t)res : 1;
    if (wpc > 8)
        wpc = 8;
    wpc = env_wpc("PCG_SCL_WPC", wpc);
    if (getenv("PCG_DEBUG_OCC"))
        fprintf(stderr, "[pcg] sclls: lds %u B, resident %d waves/CU, using %llu\n", lds, res,
                (unsigned long long)wpc);
    return (uint64_t)cus * wpc;
}

int launch_sclls(const KernelArgs& a, hipStream_t stream)
{
    const uint64_t grid = a.units;
    if (grid == 0) // no waves for a non-empty batch: an error, never a silent no-op
        return a.F ? -4 : 0;
    size_t lds = (size_t)a.wave_lds_floats * sizeof(float);
#ifdef PCG_LS_PROF
    lds += 192 * sizeof(uint64_t);
#endif
    const uint32_t lp = a.scl_lp > lp_of(a.L) ? a.scl_lp : lp_of(a.L);
#if PCG_LS_INST
    // a development build (tools/build_dev_lib.sh: this host part and one width compiled with
    // the dev knobs): the other widths' objects were built with the default knobs, whose
    // layout need not be the one computed here -- refused, never run on a mismatched layout
    if (lp != PCG_LS_INST)
        return -4;
#endif
    switch (lp) {
    case 2: return sclls_launch_2(a, lds, stream);
    case 4: return sclls_launch_4(a, lds, stream);
    case 8: return sclls_launch_8(a, lds, stream);
    case 16: return sclls_launch_16(a, lds, stream);
    case 32: return sclls_launch_32(a, lds, stream);
    default: return -4;
    }
}

#endif // PCG_LS_HOST
#endif // PCG_RTC

} // namespace pcg
