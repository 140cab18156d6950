// scl_kernel.hip -- batched CRC-aided SCL polar decoding on CDNA4 (gfx950).
//
// One codeword per wavefront (one 64-thread workgroup); the wave walks the plan's
// flattened SCL schedule (SclAvx::createDecoder order, scl_avx_float.cpp:624-651)
// for all P <= L paths at once.  The reference's PathList/DataPool lazy copies
// (scl_avx_float.cpp:21-171, datapool.txx) become:
//   * LLR stage buffers alpha[s][slot] with a per-path slot table ptr[p][s]:
//     an F/G at stage s rewrites every path's alpha[s] (all old alpha[s] are
//     dead then), so it writes slot p and resets ptr[p][s] = p; a branching leaf
//     copies ptr rows (the lazy duplicate) instead of data.  Stages below
//     `lds_stage_limit` live in LDS, the big top stages in a per-wave global
//     scratch slab (L2/MALL resident).
//   * the codeword estimate of each path as packed sign bits with in-place
//     Combine (observably identical to Bit/LeftBit stage stacks), double
//     buffered across a branching leaf.
// Candidate generation, findWeakLlrs and simplePartialSortDescending
// (arrayfuncs.h:161-231) are simulated exactly -- including their swap-induced
// tie orders -- with wave argmin/argmax reductions.
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"

namespace pcg {

namespace {

constexpr uint32_t MAXL = 32;
constexpr uint32_t MAXC = 8 * MAXL; // candidates per leaf

struct Layout {
    // float/word offsets inside one wave's LDS slice
    uint32_t alpha;  // L*(2^S_l - 1) floats
    uint32_t cw0;    // 2 * L * W words
    uint32_t ptr;    // 2 * L * 16 bytes (as words)
    uint32_t met;    // 2 * L floats
    uint32_t cval;   // MAXC floats
    uint32_t cid;    // MAXC words
    uint32_t wk;     // L * 4 floats (weak values)
    uint32_t wi;     // L * 4 words (weak indices)
    uint32_t wpar;   // L words
    uint32_t xch;    // 64 floats lane exchange
    uint32_t total;
};

// alpha slot base (in floats) of stage s inside its storage.  LDS slots are
// max(2^s, 4) floats so every stage and slot is 16-byte aligned (float4 access).
__host__ __device__ inline uint32_t lds_stage_base(uint32_t L, uint32_t s)
{
    return s == 0 ? 0u : s == 1 ? 4u * L : L * ((1u << s) + 4u);
}
__host__ __device__ inline Layout make_layout(uint32_t N, uint32_t L, uint32_t Sl)
{
    Layout y;
    const uint32_t W = N >= 32 ? N / 32 : 1;
    uint32_t o = 0;
    y.alpha = o;
    o += lds_stage_base(L, Sl);
    o = (o + 3) & ~3u;
    y.cw0 = o;
    o += 2 * L * W;
    y.ptr = o;
    o += 2 * L * 4;
    y.met = o;
    o += 2 * L;
    y.cval = o;
    o += MAXC;
    y.cid = o;
    o += MAXC;
    y.wk = o;
    o += 4 * L;
    y.wi = o;
    o += 4 * L;
    y.wpar = o;
    o += L;
    o = (o + 3) & ~3u;
    y.xch = o;
    o += 64;
    y.total = (o + 3) & ~3u;
    return y;
}

__host__ __device__ inline uint64_t gl_stage_base(uint32_t L, uint32_t s, uint32_t Sl)
{
    return (uint64_t)L * ((1ull << s) - (1ull << Sl));
}

struct Ctx {
    float* lds;             // this wave's LDS slice
    float* gs;              // this wave's global scratch slab
    const float* y;         // channel LLRs of the frame
    uint32_t N, L, top, Sl, W;
    Layout ly;
    uint32_t lane;
    uint32_t flags;         // dev-only experiment switches (PCG_FLAGS)
    bool regptr;            // L <= 8: slot table in a VGPR (lane t = stage t, 3 bits/path)
    mutable uint32_t ptrw;  // this lane's stage word of the register slot table
};

constexpr uint32_t PTR_IDENT = 0xFAC688u; // slot p for path p, 3 bits each (p = 0..7)

PCG_DEV uint8_t* ptr_tab(const Ctx& c, uint32_t cur) { return reinterpret_cast<uint8_t*>(c.lds + c.ly.ptr) + cur * c.L * 16; }
// Slot of path p at stage s (the reference's lazily shared DataPool block).
struct PtrView {
    const uint8_t* base; // LDS table column (regptr == false)
    uint32_t word;       // uniform packed stage word (regptr == true)
    bool reg;
    PCG_DEV uint32_t slot(uint32_t p) const { return reg ? (word >> (3 * p)) & 7u : base[p * 16]; }
};
PCG_DEV PtrView ptr_view(const Ctx& c, uint32_t s, uint32_t cur)
{
    PtrView v;
    v.reg = c.regptr;
    v.base = ptr_tab(c, cur) + s;
    v.word = c.regptr ? (uint32_t)__builtin_amdgcn_readlane((int)c.ptrw, (int)s) : 0u;
    return v;
}

PCG_DEV uint32_t* cw_tab(const Ctx& c, uint32_t cur) { return reinterpret_cast<uint32_t*>(c.lds + c.ly.cw0) + cur * c.L * c.W; }
PCG_DEV float* met_tab(const Ctx& c, uint32_t cur) { return c.lds + c.ly.met + cur * c.L; }

// ---- stage storage access, address space explicit ---------------------------------
struct LdsStage {
    float* b;
    uint32_t n;
    PCG_DEV float* slot(uint32_t q) const { return b + q * n; }
};
struct GlStage {
    float* b;
    uint32_t n;
    PCG_DEV float* slot(uint32_t q) const { return b + (uint64_t)q * n; }
};
struct ChanStage { // the root: channel LLRs, one "slot"
    const float* y;
    PCG_DEV const float* slot(uint32_t) const { return y; }
};

PCG_DEV LdsStage lds_stage(const Ctx& c, uint32_t s)
{
    return LdsStage{ c.lds + c.ly.alpha + lds_stage_base(c.L, s), s >= 2 ? (1u << s) : 4u };
}
PCG_DEV GlStage gl_stage(const Ctx& c, uint32_t s) { return GlStage{ c.gs + gl_stage_base(c.L, s, c.Sl), 1u << s }; }

// ---- internal ops ------------------------------------------------------------------
// F / G at stage s (node size 2^s): alpha[s-1][p] from alpha[s][ptr[p][s]].
// Flattened over (path, i); for h >= 4 each lane owns 4 consecutive i (float4), and
// up to 4 such chunks are loaded before any store so LDS latency overlaps.
template <int OPC, typename Src, typename Dst>
PCG_DEV void fg_op(const Ctx& c, Src src, Dst dst, uint32_t s, uint32_t o, uint32_t P, uint32_t cur)
{
    const uint32_t h = 1u << (s - 1), lh = s - 1;
    const PtrView pv = ptr_view(c, s, cur);
    const uint32_t* cw = cw_tab(c, cur);
    const uint32_t tot = P << lh;
    if (h >= 4) {
        for (uint32_t e0 = 4 * c.lane; e0 < tot; e0 += 4 * 256) {
            float4 xa[4], xb[4];
            uint32_t wb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t e = e0 + 256 * u;
                if (e < tot) {
                    const uint32_t p = e >> lh, i = e & (h - 1);
                    const auto* in = src.slot(s == c.top ? 0u : pv.slot(p));
                    xa[u] = *reinterpret_cast<const float4*>(in + i);
                    xb[u] = *reinterpret_cast<const float4*>(in + i + h);
                    if (OPC == OP_G)
                        wb[u] = cw[p * c.W + ((o + i) >> 5)] >> ((o + i) & 31);
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t e = e0 + 256 * u;
                if (e < tot) {
                    const uint32_t p = e >> lh, i = e & (h - 1);
                    float4 r;
                    if (OPC == OP_F) {
                        r.x = polar_f(xa[u].x, xb[u].x);
                        r.y = polar_f(xa[u].y, xb[u].y);
                        r.z = polar_f(xa[u].z, xb[u].z);
                        r.w = polar_f(xa[u].w, xb[u].w);
                    } else {
                        r.x = polar_g(xa[u].x, xb[u].x, (wb[u] & 1u) << 31);
                        r.y = polar_g(xa[u].y, xb[u].y, ((wb[u] >> 1) & 1u) << 31);
                        r.z = polar_g(xa[u].z, xb[u].z, ((wb[u] >> 2) & 1u) << 31);
                        r.w = polar_g(xa[u].w, xb[u].w, ((wb[u] >> 3) & 1u) << 31);
                    }
                    *reinterpret_cast<float4*>(dst.slot(p) + i) = r;
                }
            }
        }
    } else {
        for (uint32_t e = c.lane; e < tot; e += 64) {
            const uint32_t p = e >> lh, i = e & (h - 1);
            const auto* in = src.slot(s == c.top ? 0u : pv.slot(p));
            float r;
            if (OPC == OP_F)
                r = polar_f(in[i], in[i + h]);
            else
                r = polar_g(in[i], in[i + h], get_bit(cw + p * c.W, o + i) << 31);
            dst.slot(p)[i] = r;
        }
    }
}

template <int OPC>
PCG_DEV void fg_dispatch(const Ctx& c, uint32_t s, uint32_t o, uint32_t P, uint32_t cur)
{
    const uint32_t d = s - 1;
    if (c.flags & 2u) {
        // timing experiment only (PCG_FLAGS): skip the arithmetic
    } else if (s == c.top) {
        if (d >= c.Sl)
            fg_op<OPC>(c, ChanStage{ c.y }, gl_stage(c, d), s, o, P, cur);
        else
            fg_op<OPC>(c, ChanStage{ c.y }, lds_stage(c, d), s, o, P, cur);
    } else if (s >= c.Sl) {
        if (d >= c.Sl)
            fg_op<OPC>(c, gl_stage(c, s), gl_stage(c, d), s, o, P, cur);
        else
            fg_op<OPC>(c, gl_stage(c, s), lds_stage(c, d), s, o, P, cur);
    } else {
        fg_op<OPC>(c, lds_stage(c, s), lds_stage(c, d), s, o, P, cur);
    }
    wsync();
    // every path now owns slot p of stage d
    if (c.regptr) {
        c.ptrw = c.lane == d ? PTR_IDENT : c.ptrw;
    } else {
        uint8_t* ptr = ptr_tab(c, cur);
        for (uint32_t p = c.lane; p < P; p += 64)
            ptr[p * 16 + d] = (uint8_t)p;
    }
}

// COMB at stage s: cw[p][o+i] ^= cw[p][o+h+i], i < h
PCG_DEV void comb_op(const Ctx& c, uint32_t s, uint32_t o, uint32_t P, uint32_t cur)
{
    const uint32_t h = 1u << (s - 1);
    uint32_t* cw = cw_tab(c, cur);
    if (h >= 32) {
        const uint32_t nw = h >> 5, lw = __builtin_ctz(nw);
        const uint32_t wl = o >> 5, wr = (o + h) >> 5;
        for (uint32_t e = c.lane; e < (P << lw); e += 64) {
            const uint32_t p = e >> lw, i = e & (nw - 1);
            cw[p * c.W + wl + i] ^= cw[p * c.W + wr + i];
        }
    } else {
        const uint32_t sh = o & 31, msk = ((1u << h) - 1u) << sh;
        for (uint32_t p = c.lane; p < P; p += 64) {
            uint32_t* w = cw + p * c.W + (o >> 5);
            *w ^= (*w >> h) & msk;
        }
    }
}

// Ordered 8-lane sum ((((((s0+s1)+s2)+s3)+s4)+s5)+s6)+s7 of aligned 8-lane groups
// (reduce_add_ps, avxconvenience.h:256-272), through the wave's LDS exchange area.
// Valid in the first lane of each group.
PCG_DEV float ordered_sum8(const Ctx& c, float s)
{
    float* x = c.lds + c.ly.xch;
    x[c.lane] = s;
    wsync();
    float r = 0.0f;
    if ((c.lane & 7) == 0) {
        const float4 a = *reinterpret_cast<const float4*>(x + c.lane);
        const float4 b = *reinterpret_cast<const float4*>(x + c.lane + 4);
        r = a.x;
        r = r + a.y;
        r = r + a.z;
        r = r + a.w;
        r = r + b.x;
        r = r + b.y;
        r = r + b.z;
        r = r + b.w;
    }
    wsync();
    return r;
}

// ---- leaves --------------------------------------------------------------------------
PCG_DEV void clear_bits(const Ctx& c, uint32_t s, uint32_t o, uint32_t P, uint32_t cur);

// Rate-0 (scl_avx_float.cpp:316-337): metric += reduce_add(sum_lanes min(llr, +0)); no re-sort.
template <typename Src>
PCG_DEV void leaf_r0(const Ctx& c, Src src, uint32_t s, uint32_t o, uint32_t P, uint32_t cur)
{
    const uint32_t n = 1u << s;
    const PtrView pv = ptr_view(c, s, cur);
    float* met = met_tab(c, cur);
    for (uint32_t p0 = 0; p0 < P; p0 += 8) {
        const uint32_t p = p0 + (c.lane >> 3), j = c.lane & 7;
        float acc = 0.0f;
        if (p < P) {
            const float* in = src.slot(s == c.top ? 0u : pv.slot(p));
            if (n < 8) {
                acc = acc + minps(j < n ? in[j] : 0.0f, 0.0f);
            } else {
                for (uint32_t i = j; i < n; i += 8)
                    acc = acc + minps(in[i], 0.0f);
            }
        }
        const float pen = ordered_sum8(c, acc);
        if (p < P && j == 0)
            met[p] = met[p] + pen;
    }
    clear_bits(c, s, o, P, cur);
}

// bits [o, o+2^s) = 0 (+INF) for every path
PCG_DEV void clear_bits(const Ctx& c, uint32_t s, uint32_t o, uint32_t P, uint32_t cur)
{
    const uint32_t n = 1u << s;
    uint32_t* cw = cw_tab(c, cur);
    if (n >= 32) {
        const uint32_t nw = n >> 5, lw = __builtin_ctz(nw);
        for (uint32_t e = c.lane; e < (P << lw); e += 64)
            cw[(e >> lw) * c.W + (o >> 5) + (e & (nw - 1))] = 0u;
    } else {
        const uint32_t msk = ((1u << n) - 1u) << (o & 31);
        for (uint32_t p = c.lane; p < P; p += 64)
            cw[p * c.W + (o >> 5)] &= ~msk;
    }
}

// Repetition, n < 8 (scl_avx_float.cpp:428-481): 2 candidates per path
template <typename Src>
PCG_DEV void cand_rep(const Ctx& c, Src src, uint32_t s, uint32_t P, uint32_t cur)
{
    const uint32_t n = 1u << s;
    const PtrView pv = ptr_view(c, s, cur);
    const float* met = met_tab(c, cur);
    float* cval = c.lds + c.ly.cval;
    for (uint32_t p0 = 0; p0 < P; p0 += 8) {
        const uint32_t p = p0 + (c.lane >> 3), j = c.lane & 7;
        float l = 0.0f;
        if (p < P) {
            const float* in = src.slot(s == c.top ? 0u : pv.slot(p));
            l = j < n ? in[j] : 0.0f;
        }
        const float z = 0.0f + minps(l, 0.0f);
        const float on = 0.0f + maxps(l, 0.0f);
        const float Z = ordered_sum8(c, z);
        const float O = ordered_sum8(c, on);
        if (p < P && j == 0) {
            const float m = met[p];
            cval[2 * p] = m + Z;
            cval[2 * p + 1] = m - O;
        }
    }
}

// findWeakLlrs(idx, |llr|, n, k) (arrayfuncs.h:209-231) for every path, exact swap
// semantics, plus the SPC parity (XOR of all n signs).  Results: wk[p][0..k),
// wi[p][0..k), wpar[p].  All paths run together: groups of g lanes per path
// (g = min(n, max(64/P2, 8))), each lane scanning positions gl, gl+g, ...  The
// selection-sort swaps are tracked as an overlay of <= k displaced positions.
template <typename Src>
PCG_DEV void weak_search(const Ctx& c, Src src, uint32_t s, uint32_t P, uint32_t cur, uint32_t k)
{
    const uint32_t n = 1u << s;
    uint32_t P2 = 1;
    while (P2 < P)
        P2 <<= 1;
    uint32_t g = 64 / P2;
    if (g < 8)
        g = 8;
    if (g > n)
        g = n;
    const uint32_t lg = __builtin_ctz(g);
    const uint32_t gpp = 64 >> lg; // paths per pass
    const uint32_t gl = c.lane & (g - 1);
    const PtrView pv = ptr_view(c, s, cur);
    float* wk = c.lds + c.ly.wk;
    uint32_t* wi = reinterpret_cast<uint32_t*>(c.lds + c.ly.wi);
    uint32_t* wpar = reinterpret_cast<uint32_t*>(c.lds + c.ly.wpar);
    const uint32_t lim = (n - 1) < k ? (n - 1) : k;
    for (uint32_t p0 = 0; p0 < P; p0 += gpp) {
        const uint32_t p = p0 + (c.lane >> lg);
        const bool act = p < P;
        const float* in = src.slot(s == c.top ? 0u : pv.slot(act ? p : 0));
        uint32_t par = 0;
        if (act)
            for (uint32_t i = gl; i < n; i += g)
                par ^= fbits(in[i]);
        par = grp_xor(par, g);
        uint32_t ovp[4] = { ~0u, ~0u, ~0u, ~0u }, ovi[4] = { 0, 0, 0, 0 };
        float ovv[4] = { 0, 0, 0, 0 };
        const bool wr = act && gl == 0;
        for (uint32_t t = 0; t < lim; ++t) {
            float bv = __builtin_inff();
            uint32_t bi = 0xffffffffu;
            if (act) {
                for (uint32_t i = gl; i < n; i += g) {
                    const bool inov = (i == ovp[0]) | (i == ovp[1]) | (i == ovp[2]) | (i == ovp[3]);
                    const float v = fabs_(in[i]);
                    if (i >= t && !inov && (bi == 0xffffffffu || v < bv)) {
                        bv = v;
                        bi = i;
                    }
                }
                if (gl == 0) {
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q) {
                        if (ovp[q] != ~0u && ovp[q] >= t &&
                            (bi == 0xffffffffu || ovv[q] < bv || (ovv[q] == bv && ovp[q] < bi))) {
                            bv = ovv[q];
                            bi = ovp[q];
                        }
                    }
                }
            }
            grp_argmin(bv, bi, g);
            uint32_t bo = bi;
            float vt = 0.0f;
            uint32_t it = t;
            bool tov = false;
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                if (ovp[q] == bi)
                    bo = ovi[q];
                if (ovp[q] == t) {
                    vt = ovv[q];
                    it = ovi[q];
                    tov = true;
                }
            }
            if (wr) {
                wk[p * 4 + t] = bv;
                wi[p * 4 + t] = bo;
            }
            if (bi != t) { // the element at position t moves to position bi
                if (!tov)
                    vt = act ? fabs_(in[t]) : 0.0f;
                bool placed = false;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    if (ovp[q] == bi) {
                        ovv[q] = vt;
                        ovi[q] = it;
                        placed = true;
                    }
                if (!placed) {
#pragma unroll
                    for (uint32_t q = 0; q < 4; ++q)
                        if (q == t) { // pass t adds at most overlay entry t
                            ovp[q] = bi;
                            ovv[q] = vt;
                            ovi[q] = it;
                        }
                }
            }
        }
        // positions left after lim passes (n-1 < k)
        for (uint32_t t = lim; t < k; ++t) {
            float vt = (act && t < n) ? fabs_(in[t]) : __builtin_inff();
            uint32_t it = t;
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q)
                if (ovp[q] == t) {
                    vt = ovv[q];
                    it = ovi[q];
                }
            if (wr) {
                wk[p * 4 + t] = vt;
                wi[p * 4 + t] = it;
            }
        }
        if (wr)
            wpar[p] = par & 0x80000000u;
    }
}

// Lane-serial leaves for n <= 8 (the common case): lane p handles path p alone, in
// registers, reproducing the reference's per-path loops literally.
//   R0  : metric += reduce_add(0 + min(l_j, 0))                         :316-337
//   REP : candidates m + reduce(0 + min(l,0)), m - reduce(0 + max(l,0)) :428-481
//   R1/SPC: findWeakLlrs on |l| with its swaps, then the candidates     :353-413, 498-621
PCG_DEV void load8(const float* x, uint32_t n, float (&v)[8])
{
    // slots are 16-byte aligned and at least 4 floats wide (lds_stage_base)
    const float4 z4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float4 a = *reinterpret_cast<const float4*>(x);
    const float4 b = n >= 8 ? *reinterpret_cast<const float4*>(x + 4) : z4;
    if (n < 4) {
        a.z = 0.0f;
        a.w = 0.0f;
        if (n < 2)
            a.y = 0.0f;
    }
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

PCG_DEV float ordered8(const float (&a)[8])
{
    return a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6] + a[7];
}

PCG_DEV void small_leaf(const Ctx& c, uint32_t code, uint32_t s, uint32_t P, uint32_t cur)
{
    const uint32_t n = 1u << s, p = c.lane;
    const PtrView pv = ptr_view(c, s, cur);
    if (p >= P)
        return;
    float* met = met_tab(c, cur);
    const float* x = lds_stage(c, s).slot(pv.slot(p));
    float v[8];
    load8(x, n, v);
    const float m = met[p];
    float* cval = c.lds + c.ly.cval;
    if (code == OP_S_R0) {
        float q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            q[j] = 0.0f + minps(j < (int)n ? v[j] : 0.0f, 0.0f);
        met[p] = m + ordered8(q);
        return;
    }
    if (code == OP_S_REP) {
        float z[8], o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float l = j < (int)n ? v[j] : 0.0f;
            z[j] = 0.0f + minps(l, 0.0f);
            o[j] = 0.0f + maxps(l, 0.0f);
        }
        cval[2 * p] = m + ordered8(z);
        cval[2 * p + 1] = m - ordered8(o);
        return;
    }
    // R1 / SPC
    const uint32_t kk = code == OP_S_R1 ? 2 : 4;
    float T[8];
    uint32_t I[8];
    uint32_t par = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        T[j] = fabs_(v[j]);
        I[j] = (uint32_t)j;
        if (j < (int)n)
            par ^= fbits(v[j]);
    }
    const uint32_t lim = (n - 1) < kk ? (n - 1) : kk;
    // Selection passes with the reference's swaps.  Element updates use bit masks
    // instead of conditional array stores so the arrays stay in registers.
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (t < (int)lim) {
            float bv = T[t];
            uint32_t b = (uint32_t)t;
#pragma unroll
            for (int j = t + 1; j < 8; ++j) {
                const bool better = j < (int)n && T[j] < bv;
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
    float* wk = c.lds + c.ly.wk;
    uint32_t* wi = reinterpret_cast<uint32_t*>(c.lds + c.ly.wi);
    uint32_t* wpar = reinterpret_cast<uint32_t*>(c.lds + c.ly.wpar);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        wk[p * 4 + t] = T[t];
        wi[p * 4 + t] = I[t];
    }
    const uint32_t odd = par & 0x80000000u;
    wpar[p] = odd;
    if (code == OP_S_R1) {
        cval[4 * p] = m;
        cval[4 * p + 1] = m - T[0];
        cval[4 * p + 2] = m - T[1];
        cval[4 * p + 3] = m - T[0] - T[1];
    } else {
        float mm = m, pinv = 1.0f;
        if (odd) {
            pinv = 0.0f;
            mm -= T[0];
        }
        float* cv = cval + 8 * p;
        cv[0] = mm;
        cv[1] = mm - pinv * T[0] - T[1];
        cv[2] = mm - pinv * T[0] - T[2];
        cv[3] = mm - pinv * T[0] - T[3];
        cv[4] = mm - T[1] - T[2];
        cv[5] = mm - T[1] - T[3];
        cv[6] = mm - T[2] - T[3];
        cv[7] = mm - pinv * T[0] - T[1] - T[2] - T[3];
    }
}

// candidate metrics from the weak values (scl_avx_float.cpp:365-379 and :530-585)
PCG_DEV void cand_r1_spc(const Ctx& c, uint32_t code, uint32_t P, uint32_t cur)
{
    const float* met = met_tab(c, cur);
    const float* wk = c.lds + c.ly.wk;
    const uint32_t* wpar = reinterpret_cast<const uint32_t*>(c.lds + c.ly.wpar);
    float* cval = c.lds + c.ly.cval;
    const uint32_t k = code == OP_S_R1 ? 4 : 8;
    for (uint32_t e = c.lane; e < P * k; e += 64) {
        const uint32_t p = e / k, j = e % k;
        const float* T = wk + p * 4;
        float m = met[p];
        float v;
        if (code == OP_S_R1) {
            if (j == 0)
                v = m;
            else if (j == 1)
                v = m - T[0];
            else if (j == 2)
                v = m - T[1];
            else
                v = m - T[0] - T[1];
        } else {
            float pinv = 1.0f;
            if (wpar[p]) { // odd parity: the reference charges T0 up front
                pinv = 0.0f;
                m -= T[0];
            }
            switch (j) {
            case 0: v = m; break;
            case 1: v = m - pinv * T[0] - T[1]; break;
            case 2: v = m - pinv * T[0] - T[2]; break;
            case 3: v = m - pinv * T[0] - T[3]; break;
            case 4: v = m - T[1] - T[2]; break;
            case 5: v = m - T[1] - T[3]; break;
            case 6: v = m - T[2] - T[3]; break;
            default: v = m - pinv * T[0] - T[1] - T[2] - T[3]; break;
            }
        }
        cval[e] = v;
    }
}

// flip mask over the 4 weak indices for candidate j, one nibble per candidate:
// R1 {}, {i0}, {i1}, {i0,i1};  SPC even parity {}, {0,1}, {0,2}, {0,3}, {1,2}, {1,3},
// {2,3}, {0,1,2,3};  SPC odd parity {0}, {1}, {2}, {3}, {0,1,2}, {0,1,3}, {0,2,3}, {1,2,3}
// (scl_avx_float.cpp:375-378 and 533-585).
PCG_DEV uint32_t flip_sel(uint32_t code, uint32_t j, uint32_t oddpar)
{
    const uint32_t tab = code == OP_S_R1 ? 0x3210u : oddpar ? 0xEDB78421u : 0xFCA69530u;
    return (tab >> (4 * j)) & 0xFu;
}

// simplePartialSortDescending(idx, cval, np, C) (arrayfuncs.h:161-183): exact swap
// selection, positions held R-per-lane (pos = lane + 64 r) in named registers (no
// private arrays), DPP argmax per pass, swaps through readlane.  Leaves cval/cid[0..np).
template <int R>
PCG_DEV void partial_sort_r(const Ctx& c, uint32_t C, uint32_t np)
{
    float* cval = c.lds + c.ly.cval;
    uint32_t* cid = reinterpret_cast<uint32_t*>(c.lds + c.ly.cid);
    const uint32_t l = c.lane;
    float v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    uint32_t i0 = l, i1 = l + 64, i2 = l + 128, i3 = l + 192;
    v0 = l < C ? cval[l] : 0.0f;
    if (R > 1) {
        v1 = l + 64 < C ? cval[l + 64] : 0.0f;
        v2 = l + 128 < C ? cval[l + 128] : 0.0f;
        v3 = l + 192 < C ? cval[l + 192] : 0.0f;
    }
    const uint32_t lim = (C - 1) < np ? (C - 1) : np;
    for (uint32_t t = 0; t < lim; ++t) {
        float bv = 0.0f;
        uint32_t bp = 0xffffffffu;
        auto offer = [&](float v, uint32_t pos) {
            if (pos >= t && pos < C && (bp == 0xffffffffu || v > bv)) {
                bv = v;
                bp = pos;
            }
        };
        offer(v0, l);
        if (R > 1) {
            offer(v1, l + 64);
            offer(v2, l + 128);
            offer(v3, l + 192);
        }
        wave_argmax_dpp(bv, bp);
        const uint32_t b = __builtin_amdgcn_readfirstlane(bp);
        if (b == t)
            continue;
        const uint32_t rt = t >> 6, lt = t & 63, rb = b >> 6, lb = b & 63;
        auto rdv = [&](uint32_t r, uint32_t ln) -> float {
            float x = ubits((uint32_t)__builtin_amdgcn_readlane((int)fbits(v0), (int)ln));
            if (R > 1) {
                const float x1 = ubits((uint32_t)__builtin_amdgcn_readlane((int)fbits(v1), (int)ln));
                const float x2 = ubits((uint32_t)__builtin_amdgcn_readlane((int)fbits(v2), (int)ln));
                const float x3 = ubits((uint32_t)__builtin_amdgcn_readlane((int)fbits(v3), (int)ln));
                x = r == 1 ? x1 : r == 2 ? x2 : r == 3 ? x3 : x;
            }
            return x;
        };
        auto rdi = [&](uint32_t r, uint32_t ln) -> uint32_t {
            uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)i0, (int)ln);
            if (R > 1) {
                const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)i1, (int)ln);
                const uint32_t x2 = (uint32_t)__builtin_amdgcn_readlane((int)i2, (int)ln);
                const uint32_t x3 = (uint32_t)__builtin_amdgcn_readlane((int)i3, (int)ln);
                x = r == 1 ? x1 : r == 2 ? x2 : r == 3 ? x3 : x;
            }
            return x;
        };
        const float vt = rdv(rt, lt), vb = rdv(rb, lb);
        const uint32_t it = rdi(rt, lt), ib = rdi(rb, lb);
        const bool at_t = l == lt, at_b = l == lb;
        if (rt == 0 && at_t) { v0 = vb; i0 = ib; }
        if (rb == 0 && at_b) { v0 = vt; i0 = it; }
        if (R > 1) {
            if (rt == 1 && at_t) { v1 = vb; i1 = ib; }
            if (rb == 1 && at_b) { v1 = vt; i1 = it; }
            if (rt == 2 && at_t) { v2 = vb; i2 = ib; }
            if (rb == 2 && at_b) { v2 = vt; i2 = it; }
            if (rt == 3 && at_t) { v3 = vb; i3 = ib; }
            if (rb == 3 && at_b) { v3 = vt; i3 = it; }
        }
    }
    if (l < np) {
        cval[l] = v0;
        cid[l] = i0;
    }
    if (R > 1) {
        if (l + 64 < np) { cval[l + 64] = v1; cid[l + 64] = i1; }
        if (l + 128 < np) { cval[l + 128] = v2; cid[l + 128] = i2; }
        if (l + 192 < np) { cval[l + 192] = v3; cid[l + 192] = i3; }
    }
}

// One bitonic compare-exchange of (value, id) with the exact xor-J partner; `keep_max`
// says whether this lane keeps the larger value.
template <int J>
PCG_DEV void bitonic_cx(float& v, uint32_t& id, bool keep_max)
{
    const float ov = ubits(xpartner<J>(fbits(v)));
    const uint32_t oi = xpartner<J>(id);
    const bool take = keep_max ? (ov > v) : (ov < v);
    if (take) {
        v = ov;
        id = oi;
    }
}

template <int K, int J>
PCG_DEV void bitonic_stage(float& v, uint32_t& id, uint32_t l)
{
    const bool desc = (K == 64) || ((l & K) == 0);
    const bool lower = (l & J) == 0;
    bitonic_cx<J>(v, id, lower == desc);
}

// Fast path for C <= 64 candidates: full bitonic sort (descending) across the wave.
// When the np+1 leading values are pairwise distinct, swap-selection produces exactly
// this order; otherwise (ties) the exact swap-selection simulation runs instead.
PCG_DEV void partial_sort(const Ctx& c, uint32_t C, uint32_t np)
{
    if (C > 64) {
        partial_sort_r<4>(c, C, np);
        return;
    }
    float* cval = c.lds + c.ly.cval;
    uint32_t* cid = reinterpret_cast<uint32_t*>(c.lds + c.ly.cid);
    const uint32_t l = c.lane;
    float v = l < C ? cval[l] : -__builtin_inff();
    uint32_t id = l;
    bitonic_stage<2, 1>(v, id, l);
    bitonic_stage<4, 2>(v, id, l);
    bitonic_stage<4, 1>(v, id, l);
    bitonic_stage<8, 4>(v, id, l);
    bitonic_stage<8, 2>(v, id, l);
    bitonic_stage<8, 1>(v, id, l);
    bitonic_stage<16, 8>(v, id, l);
    bitonic_stage<16, 4>(v, id, l);
    bitonic_stage<16, 2>(v, id, l);
    bitonic_stage<16, 1>(v, id, l);
    bitonic_stage<32, 16>(v, id, l);
    bitonic_stage<32, 8>(v, id, l);
    bitonic_stage<32, 4>(v, id, l);
    bitonic_stage<32, 2>(v, id, l);
    bitonic_stage<32, 1>(v, id, l);
    bitonic_stage<64, 32>(v, id, l);
    bitonic_stage<64, 16>(v, id, l);
    bitonic_stage<64, 8>(v, id, l);
    bitonic_stage<64, 4>(v, id, l);
    bitonic_stage<64, 2>(v, id, l);
    bitonic_stage<64, 1>(v, id, l);
    // next lane's value (wave_shl:1 = lane i reads lane i+1)
    const float vn = ubits((uint32_t)__builtin_amdgcn_update_dpp((int)fbits(v), (int)fbits(v), 0x130, 0xF, 0xF, false));
    const uint32_t last = (np < C) ? np : (C - 1); // compare positions i, i+1 for i < last
    const bool tie = (l < last) && (v == vn);
    if (ballot(tie) != 0ull) {
        partial_sort_r<1>(c, C, np);
        return;
    }
    if (l < np) {
        cval[l] = v;
        cid[l] = id;
    }
}

// Build the next path list after a branching leaf: duplicate (ptr rows + codeword
// words up to the leaf's end), set metrics, write the leaf's bits.
template <typename Src>
PCG_DEV void branch_commit(const Ctx& c, Src src, uint32_t code, uint32_t s, uint32_t o, uint32_t P,
                           uint32_t np, uint32_t k, uint32_t cur)
{
    const uint32_t n = 1u << s, nxt = cur ^ 1u;
    const uint8_t* ptr = ptr_tab(c, cur);
    uint8_t* ptr2 = ptr_tab(c, nxt);
    const uint32_t* cw = cw_tab(c, cur);
    uint32_t* cw2 = cw_tab(c, nxt);
    float* met2 = met_tab(c, nxt);
    const float* cval = c.lds + c.ly.cval;
    const uint32_t* cid = reinterpret_cast<const uint32_t*>(c.lds + c.ly.cid);
    const uint32_t* wi = reinterpret_cast<const uint32_t*>(c.lds + c.ly.wi);
    const uint32_t* wpar = reinterpret_cast<const uint32_t*>(c.lds + c.ly.wpar);
    // codeword words [0, ceil((o+n)/32)) and ptr rows
    const uint32_t nw = (o + n + 31) >> 5;
    for (uint32_t e = c.lane; e < np * nw; e += 64) {
        const uint32_t q = e / nw, w = e % nw;
        const uint32_t srcp = cid[q] / k;
        cw2[q * c.W + w] = cw[srcp * c.W + w];
    }
    const PtrView pv = ptr_view(c, s, cur); // the leaf's own stage, read before the table changes
    if (c.regptr) {
        uint32_t nw2 = 0;
        for (uint32_t q = 0; q < np; ++q)
            nw2 |= ((c.ptrw >> (3 * (cid[q] / k))) & 7u) << (3 * q);
        c.ptrw = nw2;
    } else {
        for (uint32_t e = c.lane; e < np * 4; e += 64) {
            const uint32_t q = e >> 2, w = e & 3;
            reinterpret_cast<uint32_t*>(ptr2)[q * 4 + w] = reinterpret_cast<const uint32_t*>(ptr)[(cid[q] / k) * 4 + w];
        }
    }
    for (uint32_t q = c.lane; q < np; q += 64)
        met2[q] = cval[q];
    wsync();
    // leaf bits into [o, o+n) of each survivor
    const uint32_t g = n < 64 ? n : 64;
    const uint32_t lg = __builtin_ctz(g);
    const uint32_t gpp = 64 >> lg;
    for (uint32_t q0 = 0; q0 < np; q0 += gpp) {
        const uint32_t q = q0 + (c.lane >> lg), gl = c.lane & (g - 1);
        const bool act = q < np;
        uint32_t srcp = 0, j = 0, fm = 0;
        uint32_t wq[4] = { 0, 0, 0, 0 };
        if (act) {
            srcp = cid[q] / k;
            j = cid[q] % k;
            if (code != OP_S_REP) {
                fm = flip_sel(code, j, wpar[srcp]);
                for (uint32_t t = 0; t < 4; ++t)
                    wq[t] = wi[srcp * 4 + t];
            }
        }
        const float* in = src.slot(s == c.top ? 0u : pv.slot(act ? srcp : 0));
        for (uint32_t b = 0; b < n; b += g) {
            const uint32_t i = b + gl;
            uint32_t bit = 0;
            if (act) {
                if (code == OP_S_REP) {
                    bit = j; // +|S| -> 0, -|S| -> 1 (also for S == 0: -0.0)
                } else {
                    bit = sgn(in[i]) >> 31;
                    for (uint32_t t = 0; t < 4; ++t)
                        if (((fm >> t) & 1u) && wq[t] == i)
                            bit ^= 1u;
                }
            }
            const uint64_t m = ballot(bit != 0);
            if (g >= 32) {
                // g = 32 or 64: whole words; lane 0 of each 32-lane half writes
                const uint32_t half = c.lane >> 5;
                if ((c.lane & 31) == 0 && act && (g == 64 || true)) {
                    const uint32_t wv = (uint32_t)(m >> (32 * half));
                    const uint32_t pos = o + b + (g == 64 ? 32 * half : 0);
                    cw2[q * c.W + (pos >> 5)] = wv;
                }
            } else if (gl == 0 && act) {
                const uint32_t grp = c.lane >> lg;
                const uint32_t field = (uint32_t)(m >> (grp * g)) & ((1u << g) - 1u);
                const uint32_t sh = (o + b) & 31, msk = ((1u << g) - 1u) << sh;
                uint32_t* w = cw2 + q * c.W + ((o + b) >> 5);
                *w = (*w & ~msk) | (field << sh);
            }
        }
    }
}

PCG_DEV void write_bits_from_info(const Ctx& c, const KernelArgs& a, const uint32_t* bits, uint64_t frame, bool write,
                                  uint32_t* syn)
{
    uint32_t sv = 0;
    for (uint32_t b = c.lane; b < a.kb; b += 64) {
        uint32_t byte = 0;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t idx = 8 * b + j;
            if (idx < a.K) {
                const uint32_t bit = get_bit(bits, a.info_pos[idx]);
                byte |= bit << (7 - j);
                if (bit)
                    sv ^= a.crc_m[idx];
            }
        }
        if (write)
            a.info[frame * a.kb + b] = (uint8_t)byte;
    }
    *syn = wave_xor(sv) ^ a.crc_c0;
}

// ======================= ST8: a size-8 subtree, lane = path, in registers ==========
// Runs RateR(8) -> {R0, R1, Rep, SPC, RateR(4) -> {R0, R1, Rep}} exactly as the
// reference's ShortRateRNode recursion (scl_avx_float.cpp:273-307) and leaves
// (:316-621) for every path at once, keeping the size-8 input, the size-4 input and
// the 8 codeword bits of each path in its lane's registers.  A branching leaf
// gathers the candidates, runs the same exact selection as the other leaves and
// moves the survivors' register state with ds_bpermute; the LDS path state
// (codeword prefix, slot table) is duplicated once, at the end of the subtree, from
// the path each survivor descends from.
struct St8 {
    float x8[8];
    float a4[4];
    uint32_t bits; // bit i = codeword position o + i
    uint32_t root; // path index at subtree entry
    float m;
    uint32_t P;
    bool branched;
};

// lane-serial candidates of a leaf of size n (2 or 4) on v[0..n): values cv[0..k) and
// per-candidate n-bit patterns packed 4 bits each into pat.
PCG_DEV void st_cands(uint32_t kind, const float (&v)[4], uint32_t n, float m, float (&cv)[8], uint32_t& pat)
{
    const uint32_t nmask = (1u << n) - 1u;
    if (kind == ST_REP) { // :428-481 (zero padded to 8 lanes)
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
    if (kind == ST_R1) { // :365-379
        cv[0] = m;
        cv[1] = m - T[0];
        cv[2] = m - T[1];
        cv[3] = m - T[0] - T[1];
        pat = base | ((base ^ ib[0]) << 4) | ((base ^ ib[1]) << 8) | ((base ^ ib[0] ^ ib[1]) << 12);
        return;
    }
    // SPC (n = 4): :511-585
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
        const uint32_t fm = flip_sel(OP_S_SPC, j, odd ? 1u : 0u);
        uint32_t fl = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            fl |= ((fm >> q) & 1u) ? ib[q] : 0u;
        pat |= ((base ^ fl) & nmask) << (4 * j);
    }
}

PCG_DEV void st_r0(St8& st, const float (&v)[4], uint32_t n)
{
    float q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        q[j] = 0.0f + minps(j < (int)n && j < 4 ? v[j & 3] : 0.0f, 0.0f);
    st.m = st.m + ordered8(q);
}

PCG_DEV void st_branch(const Ctx& c, St8& st, uint32_t kind, const float (&v)[4], uint32_t n, uint32_t boff)
{
    const uint32_t k = kind == ST_R1 ? 4u : kind == ST_SPC ? 8u : 2u;
    const uint32_t lk = kind == ST_R1 ? 2u : kind == ST_SPC ? 3u : 1u;
    float cv[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
    uint32_t pat = 0;
    st_cands(kind, v, n, st.m, cv, pat);
    float* cval = c.lds + c.ly.cval;
    if (c.lane < st.P) {
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
            if (j < k)
                cval[c.lane * k + j] = cv[j];
    }
    wsync();
    const uint32_t C = st.P * k;
    const uint32_t np = C < c.L ? C : c.L;
    partial_sort(c, C, np);
    wsync();
    const uint32_t* cid = reinterpret_cast<const uint32_t*>(c.lds + c.ly.cid);
    const uint32_t q = c.lane;
    const uint32_t id = q < np ? cid[q] : 0u;
    const float val = q < np ? cval[q] : 0.0f;
    const int src = (int)(id >> lk);
    const uint32_t j = id & (k - 1u);
#pragma unroll
    for (int i = 0; i < 8; ++i)
        st.x8[i] = shfl(st.x8[i], src);
#pragma unroll
    for (int i = 0; i < 4; ++i)
        st.a4[i] = shfl(st.a4[i], src);
    st.bits = shfl(st.bits, src);
    st.root = shfl(st.root, src);
    pat = shfl(pat, src);
    st.bits |= ((pat >> (4 * j)) & ((1u << n) - 1u)) << boff;
    st.m = val;
    st.P = np;
    st.branched = true;
}

PCG_DEV void st_child2(const Ctx& c, St8& st, uint32_t kind, const float (&a2)[4], uint32_t boff)
{
    if (kind == ST_R0)
        st_r0(st, a2, 2);
    else
        st_branch(c, st, kind, a2, 2, boff);
}

PCG_DEV void st_child4(const Ctx& c, St8& st, uint32_t d, uint32_t boff)
{
    const uint32_t kind = d & 7u;
    if (kind == ST_R0) {
        st_r0(st, st.a4, 4);
    } else if (kind != ST_RATER) {
        const float v[4] = { st.a4[0], st.a4[1], st.a4[2], st.a4[3] };
        st_branch(c, st, kind, v, 4, boff);
    } else { // ShortRateRNode(4): F, left(2), G, right(2), CombineBitsShort
        float a2[4] = { polar_f(st.a4[0], st.a4[2]), polar_f(st.a4[1], st.a4[3]), 0.0f, 0.0f };
        st_child2(c, st, (d >> 3) & 3u, a2, boff);
        a2[0] = polar_g(st.a4[0], st.a4[2], ((st.bits >> boff) & 1u) << 31);
        a2[1] = polar_g(st.a4[1], st.a4[3], ((st.bits >> (boff + 1)) & 1u) << 31);
        st_child2(c, st, (d >> 5) & 3u, a2, boff + 2);
        st.bits ^= ((st.bits >> (boff + 2)) & 3u) << boff;
    }
}

template <typename Src>
PCG_DEV void st8_run(const Ctx& c, Src src, uint32_t desc, uint32_t o, uint32_t& P, uint32_t& cur)
{
    const uint8_t* ptr = ptr_tab(c, cur);
    const PtrView pv = ptr_view(c, 3, cur);
    float* met = met_tab(c, cur);
    St8 st;
    st.P = P;
    st.branched = false;
    st.root = c.lane;
    st.bits = 0;
    const uint32_t p = c.lane < P ? c.lane : 0u;
    {
        const float* x = src.slot(c.top == 3 ? 0u : pv.slot(p));
        const float4 lo = *reinterpret_cast<const float4*>(x);
        const float4 hi = *reinterpret_cast<const float4*>(x + 4);
        st.x8[0] = lo.x; st.x8[1] = lo.y; st.x8[2] = lo.z; st.x8[3] = lo.w;
        st.x8[4] = hi.x; st.x8[5] = hi.y; st.x8[6] = hi.z; st.x8[7] = hi.w;
    }
    st.m = met[p];
    // F(8) -> left child (4)
#pragma unroll
    for (int i = 0; i < 4; ++i)
        st.a4[i] = polar_f(st.x8[i], st.x8[i + 4]);
    st_child4(c, st, desc & 0xffu, 0);
    // G(8) -> right child (4)
#pragma unroll
    for (int i = 0; i < 4; ++i)
        st.a4[i] = polar_g(st.x8[i], st.x8[i + 4], ((st.bits >> i) & 1u) << 31);
    st_child4(c, st, (desc >> 8) & 0xffu, 4);
    st.bits ^= (st.bits >> 4) & 0xFu; // CombineBitsShort(4)
    // write back: metrics, codeword bits [o, o+8), lazy duplicate of the LDS path state
    const uint32_t sh = o & 31u, wo = o >> 5, msk = 0xFFu << sh;
    if (!st.branched) {
        if (c.lane < P) {
            met[c.lane] = st.m;
            uint32_t* w = cw_tab(c, cur) + c.lane * c.W + wo;
            *w = (*w & ~msk) | (st.bits << sh);
        }
        return;
    }
    const uint32_t nxt = cur ^ 1u, NP = st.P, nw = wo + 1;
    const uint32_t* cw = cw_tab(c, cur);
    uint32_t* cw2 = cw_tab(c, nxt);
    const uint32_t* pt = reinterpret_cast<const uint32_t*>(ptr);
    uint32_t* pt2 = reinterpret_cast<uint32_t*>(ptr_tab(c, nxt));
    // survivors' roots and bits through the exchange area (every lane then reads them)
    uint32_t* xr = reinterpret_cast<uint32_t*>(c.lds + c.ly.xch);
    if (c.lane < NP) {
        xr[c.lane] = st.root;
        xr[32 + c.lane] = st.bits;
    }
    wsync();
    for (uint32_t e = c.lane; e < NP * nw; e += 64) {
        const uint32_t q = e / nw, w = e - q * nw;
        uint32_t v = cw[xr[q] * c.W + w];
        if (w == wo)
            v = (v & ~msk) | (xr[32 + q] << sh);
        cw2[q * c.W + w] = v;
    }
    if (c.regptr) {
        uint32_t nw2 = 0;
        for (uint32_t q = 0; q < NP; ++q)
            nw2 |= ((c.ptrw >> (3 * xr[q])) & 7u) << (3 * q);
        c.ptrw = nw2;
    } else {
        for (uint32_t e = c.lane; e < NP * 4; e += 64) {
            const uint32_t q = e >> 2;
            pt2[q * 4 + (e & 3)] = pt[xr[q] * 4 + (e & 3)];
        }
    }
    if (c.lane < NP)
        met_tab(c, nxt)[c.lane] = st.m;
    cur = nxt;
    P = NP;
}

template <typename Fn>
PCG_DEV void with_src(const Ctx& c, uint32_t s, Fn&& fn)
{
    if (s == c.top)
        fn(ChanStage{ c.y });
    else if (s >= c.Sl)
        fn(gl_stage(c, s));
    else
        fn(lds_stage(c, s));
}

} // namespace

__global__ void __launch_bounds__(64) scl_kernel(KernelArgs a)
{
    extern __shared__ float smem[];
#ifdef PCG_SPECIAL
    unsigned long long* const prof = nullptr;
#else
    unsigned long long* const prof = a.prof;
#endif
    Ctx c;
    c.lds = smem;
#ifdef PCG_SPECIAL
    c.N = 1024; c.L = 8; c.top = 10; c.Sl = 7; c.W = 32;
    c.ly = make_layout(1024, 8, 7);
#else
    c.N = a.N;
    c.L = a.L;
    c.top = a.log2N;
    c.Sl = a.lds_stage_limit;
    c.W = a.N >= 32 ? a.N / 32 : 1;
    c.ly = make_layout(a.N, a.L, a.lds_stage_limit);
#endif
    c.lane = threadIdx.x;
#ifdef PCG_SPECIAL
    c.regptr = true;
    c.flags = 0;
#else
    c.regptr = a.L <= 8 && !(a.flags & 1u);
    c.flags = a.flags;
#endif
    c.ptrw = PTR_IDENT;
    c.gs = a.scratch ? a.scratch + (uint64_t)blockIdx.x * a.scratch_floats : nullptr;

    for (uint64_t frame = blockIdx.x; frame < a.F; frame += gridDim.x) {
        c.y = a.llr + frame * a.N;
        uint32_t cur = 0, P = 1;
        if (c.lane == 0)
            met_tab(c, 0)[0] = 0.0f; // a freshly constructed decoder
        wsync();
        for (uint32_t kop = 0; kop < a.nops; ++kop) {
            // readfirstlane keeps the schedule walk wave-uniform, so ops are s_load'ed
            const uint32_t w = ld_const(a.ops, kop);
            const uint32_t code = op_code(w), s = op_stage(w), o = op_off(w);
            const uint64_t t0 = prof ? __builtin_amdgcn_s_memtime() : 0;
            switch (code) {
            case OP_F:
                fg_dispatch<OP_F>(c, s, o, P, cur);
                break;
            case OP_G:
                fg_dispatch<OP_G>(c, s, o, P, cur);
                break;
            case OP_COMB:
                if (!(c.flags & 32u))
                    comb_op(c, s, o, P, cur);
                break;
            case OP_S_ST8: {
                const uint32_t desc = ld_const(a.ops, ++kop);
                if (c.flags & 8u)
                    break;
                if (c.top == 3)
                    st8_run(c, ChanStage{ c.y }, desc, o, P, cur);
                else
                    st8_run(c, lds_stage(c, 3), desc, o, P, cur);
                break;
            }
            case OP_S_R0:
                if (c.flags & 128u)
                    break;
                if (s <= 3 && s < c.Sl && s != c.top) {
                    small_leaf(c, OP_S_R0, s, P, cur);
                    wsync();
                    clear_bits(c, s, o, P, cur);
                } else {
                    with_src(c, s, [&](auto src) { leaf_r0(c, src, s, o, P, cur); });
                }
                break;
            default: { // branching leaves
                if (c.flags & 16u)
                    break;
                const uint32_t k = code == OP_S_R1 ? 4 : code == OP_S_SPC ? 8 : 2;
                auto stamp = [&](uint32_t ph, uint64_t& tp) {
                    if (prof) {
                        const uint64_t tn = __builtin_amdgcn_s_memtime();
                        if (c.lane == 0)
                            atomicAdd(&prof[2 * ph], (unsigned long long)(tn - tp));
                        tp = tn;
                    }
                };
                uint64_t tp = t0;
                if (s <= 3 && s < c.Sl && s != c.top) {
                    small_leaf(c, code, s, P, cur);
                } else if (code == OP_S_REP) {
                    with_src(c, s, [&](auto src) { cand_rep(c, src, s, P, cur); });
                } else {
                    with_src(c, s, [&](auto src) { weak_search(c, src, s, P, cur, code == OP_S_R1 ? 2 : 4); });
                    wsync();
                    stamp(48, tp);
                    cand_r1_spc(c, code, P, cur);
                }
                wsync();
                stamp(49, tp);
                const uint32_t C = P * k;
                const uint32_t np = C < c.L ? C : c.L;
                if (c.flags & 4u) {
                    if (c.lane < np)
                        reinterpret_cast<uint32_t*>(c.lds + c.ly.cid)[c.lane] = c.lane;
                } else {
                    partial_sort(c, C, np);
                }
                wsync();
                stamp(50, tp);
                with_src(c, s, [&](auto src) { branch_commit(c, src, code, s, o, P, np, k, cur); });
                wsync();
                stamp(51, tp);
                cur ^= 1u;
                P = np;
                break;
            }
            }
            wsync();
            if (prof) {
                const uint64_t t1 = __builtin_amdgcn_s_memtime();
                if (c.lane == 0) {
                    atomicAdd(&prof[2 * code], (unsigned long long)(t1 - t0));
                    atomicAdd(&prof[2 * code + 1], 1ull);
                }
            }
        }
        // extractBestPath (scl_avx_float.cpp:711-750): first path in list order whose
        // detector check passes, else path 0.
        uint32_t* cwc = cw_tab(c, cur);
        if (!a.systematic) {
            // re-encode every path in place (G_N is applied per path)
            for (uint32_t e = c.lane; e < P * c.W; e += 64)
                cwc[e] = transform_word(cwc[e], c.N);
            wsync();
            for (uint32_t d = 1; d < c.W; d <<= 1) {
                for (uint32_t e = c.lane; e < P * c.W; e += 64) {
                    const uint32_t wi2 = e % c.W;
                    if (!(wi2 & d))
                        cwc[e] ^= cwc[e + d];
                }
                wsync();
            }
        }
        uint32_t chosen = 0, found = 0;
        for (uint32_t p = 0; p < P && !(c.flags & 64u); ++p) {
            uint32_t syn;
            write_bits_from_info(c, a, cwc + p * c.W, frame, false, &syn);
            if (syn == 0) {
                chosen = p;
                found = 1;
                break;
            }
        }
        uint32_t dummy;
        write_bits_from_info(c, a, cwc + chosen * c.W, frame, true, &dummy);
        if (c.lane == 0 && a.ok)
            a.ok[frame] = (uint8_t)found;
        if (a.metrics) {
            const float* met = met_tab(c, cur);
            for (uint32_t p = c.lane; p < c.L; p += 64)
                a.metrics[frame * c.L + p] = p < P ? met[p] : 0.0f;
        }
        wsync();
    }
}

int scl_layout(uint32_t N, uint32_t L, uint32_t* wave_lds_floats, uint32_t* lds_stage_limit, uint64_t* scratch_floats)
{
    if (L < 2 || L > MAXL)
        return -4;
    const uint32_t top = (uint32_t)__builtin_ctz(N);
    // Largest LDS-resident stage set within the budget; the rest goes to global scratch.
    uint32_t budget = 10 * 1024 / 4; // floats per wave (~16 codewords per CU)
    if (const char* e = getenv("PCG_SCL_LDS_KB"))
        budget = (uint32_t)atoi(e) * 1024 / 4;
    uint32_t Sl = top;
    const uint32_t Smin = top < 4 ? top : 4; // ST8 reads stage 3 from LDS
    while (Sl > Smin && make_layout(N, L, Sl).total > budget)
        --Sl;
    if (const char* e = getenv("PCG_SCL_STAGE_LIMIT")) {
        uint32_t v = (uint32_t)atoi(e);
        if (v >= 1 && v <= top)
            Sl = v;
    }
    const Layout ly = make_layout(N, L, Sl);
    if (ly.total * 4 > 160 * 1024)
        return -4;
    *wave_lds_floats = ly.total;
    *lds_stage_limit = Sl;
    *scratch_floats = (uint64_t)L * ((1ull << top) - (1ull << Sl));
    return 0;
}

static uint64_t g_resident_cap = 0;

uint64_t scl_scratch_frames(uint64_t F)
{
    if (g_resident_cap == 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess)
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        uint64_t wpc = 16;
        if (const char* e = getenv("PCG_SCL_WPC"))
            wpc = (uint64_t)atoi(e);
        g_resident_cap = (uint64_t)cus * wpc; // grid cap (grid-stride over frames)
    }
    return F < g_resident_cap ? F : g_resident_cap;
}

int launch_scl(const KernelArgs& a, hipStream_t stream)
{
    const uint64_t grid = scl_scratch_frames(a.F);
    if (grid == 0)
        return 0;
    const size_t lds = (size_t)a.wave_lds_floats * sizeof(float);
    hipLaunchKernelGGL(scl_kernel, dim3((uint32_t)grid), dim3(64), lds, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

} // namespace pcg
