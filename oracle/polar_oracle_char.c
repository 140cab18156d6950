/*
 * polar_oracle_char.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C scalar restatement of the reference's 8-bit fixed-point ("char")
 * decoders, the checker for the HIP int8 path:
 *   FastSscFipChar   src/polarcode/decoding/fastssc_fip_char.cpp,
 *                    include/polarcode/decoding/fip_char.h
 *   SclFipChar       src/polarcode/decoding/scl_fip_char.cpp
 *   float -> int8    CharContainer::insertLlr, src/polarcode/bitcontainer.cpp:34-39, 449-516
 * as the reference's AVX2 build computes them (BYTESPERVECTOR = 32,
 * include/polarcode/avxconvenience.h:51-53): byte-wise saturating arithmetic, the
 * 32-lane vector padding of short nodes, the reduction trees of
 * reduce_adds_epi8 / half_reduce_adds_epi8 (avxconvenience.h:92-212) and the
 * tie behaviour of minpos_epu8 (src/polarcode/avxconvenience.cpp:13-55).
 * Short-node vector operations are emulated over all 32 lanes, garbage lanes
 * included, so the memory state matches the reference's byte for byte.
 *
 * Like polar_oracle.c it is loaded only by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg (oracle/liboracle.so).  Pinned by
 * tests/test_oracle_char.py against fixtures of the reference build
 * (tests/golden/char_fixtures.npz, tests/golden/make_golden_char.py) and, where
 * oracle/_ref exists, against the live reference.
 *
 * One input class is left undefined, as it is in the reference: a 32-byte
 * vector whose 32 values are all -128 reaching minpos_epu8 (SPC / ZeroSPC
 * leaves) makes the reference read p[4] out of bounds (avxconvenience.cpp:46-48);
 * here the first lane is returned.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BV 32 /* BYTESPERVECTOR (AVX2) */

int orc_crc(int crc, int generate, uint8_t* data, int bytes); /* polar_oracle.c */

/* ------------------------------------------------------------------ */
/* byte arithmetic (_mm256_*_epi8)                                      */
/* ------------------------------------------------------------------ */
static inline int8_t sat8(int v) { return (int8_t)(v < -128 ? -128 : v > 127 ? 127 : v); }
static inline int8_t adds8(int8_t a, int8_t b) { return sat8((int)a + (int)b); }
static inline int8_t subs8(int8_t a, int8_t b) { return sat8((int)a - (int)b); }
static inline int8_t max8(int8_t a, int8_t b) { return a > b ? a : b; }
static inline int8_t min8(int8_t a, int8_t b) { return a < b ? a : b; }
/* _mm256_abs_epi8: |-128| = 0x80 (= -128 as a signed byte) */
static inline int8_t abs8(int8_t a) { return a == -128 ? (int8_t)-128 : (int8_t)(a < 0 ? -a : a); }
/* char negation as the reference writes it (BitPtr[i] = -BitPtr[i]): -(-128) stays -128 */
static inline int8_t neg8(int8_t a) { return (int8_t)(uint8_t)(0u - (uint8_t)a); }

/* FastSscFip::F_function_calc, fip_char.h:35-56 */
static inline int8_t fip_f(int8_t l, int8_t r)
{
    const int8_t x = (int8_t)((l ^ r) | 1);
    int8_t a = abs8(max8(l, -127)), b = abs8(max8(r, -127));
    a = max8(a, 1);
    b = max8(b, 1);
    const int8_t m = min8(a, b);
    return x < 0 ? (int8_t)-m : m; /* _mm256_sign_epi8, x never 0 */
}
/* G_function_calc, fip_char.h:58-64: blendv(R + L, R - L, bit) */
static inline int8_t fip_g(int8_t l, int8_t r, int8_t bit) { return bit < 0 ? subs8(r, l) : adds8(r, l); }

/* subVectorShiftBytes_epu8 / subVectorBackShiftBytes_epu8 (avxconvenience.cpp:86-148):
 * per 2h-byte group, right[i] = left[i + h] in the lower half (zeros above);
 * back[i] = x[i - h] in the upper half (zeros below). */
static void vshift(const int8_t* x, int8_t* out, unsigned h)
{
    for (unsigned i = 0; i < BV; ++i) out[i] = (i % (2 * h) < h) ? x[i + h] : 0;
}
static void vbackshift(const int8_t* x, int8_t* out, unsigned h)
{
    for (unsigned i = 0; i < BV; ++i) out[i] = (i % (2 * h) >= h) ? x[i - h] : 0;
}

/* reduce_adds_epi8 (avxconvenience.h:92-101): saturating tree, pairs (i, i+16), (i, i+8), ... */
static int8_t reduce_adds(const int8_t* x)
{
    int8_t v[BV];
    memcpy(v, x, BV);
    for (unsigned k = BV / 2; k >= 1; k >>= 1)
        for (unsigned i = 0; i < k; ++i) v[i] = adds8(v[i], v[i + k]);
    return v[0];
}
/* half_reduce_adds_epi8 (avxconvenience.h:202-212): XOR butterflies 16, 8, 4, 2 */
static void half_reduce_adds(const int8_t* x, int8_t* out)
{
    int8_t v[BV], t[BV];
    memcpy(v, x, BV);
    for (unsigned k = 16; k >= 2; k >>= 1) {
        for (unsigned i = 0; i < BV; ++i) t[i] = adds8(v[i], v[i ^ k]);
        memcpy(v, t, BV);
    }
    memcpy(out, v, BV);
}
static uint8_t reduce_xor(const int8_t* x)
{
    uint8_t r = 0;
    for (unsigned i = 0; i < BV; ++i) r ^= (uint8_t)x[i];
    return r;
}
/* minpos_epu8 (avxconvenience.cpp:13-55): first lane of the smallest unsigned byte;
 * *val = that byte as a (signed) char.  All-0x80 input: undefined in the reference. */
static unsigned minpos_epu8(const int8_t* x, int8_t* val)
{
    unsigned best = 0;
    for (unsigned i = 1; i < BV; ++i)
        if ((uint8_t)x[i] < (uint8_t)x[best]) best = i;
    if ((uint8_t)x[best] == 0x80u) best = 0; /* undefined in the reference */
    if (val) *val = x[best];
    return best;
}

/* ------------------------------------------------------------------ */
/* float -> int8 quantisation, CharContainer::insertLlr                 */
/* ------------------------------------------------------------------ */
/* convert_f32_to_int8_large (bitcontainer.cpp:468-503), n >= 32: _mm256_cvtps_epi32
 * (round to nearest even; NaN / |x| >= 2^31 -> INT32_MIN) then packs_epi32 / packs_epi16. */
static int8_t f2c_large(float x)
{
    if (x != x || x >= 2147483648.0f || x < -2147483648.0f) return -128;
    const float r = rintf(x);
    return r <= -128.0f ? (int8_t)-128 : r >= 127.0f ? (int8_t)127 : (int8_t)(int)r;
}
/* vectorizedFtoC (:449-466), 8 <= n < 32: max(x,-128) (NaN -> -128), min(.,127), round to
 * nearest even, low byte of the int32 */
static int8_t f2c_vec(float x)
{
    float v = x > -128.0f ? x : -128.0f;
    v = v < 127.0f ? v : 127.0f;
    return (int8_t)(int)rintf(v);
}
/* convertFtoC (:34-39), n < 8: fmin(fmax(x,-128),127) then round() (half away from zero) */
static int8_t f2c_scalar(float x)
{
    return (int8_t)(int)roundf(fminf(fmaxf(x, -128.0f), 127.0f));
}

void orc_f32_to_i8(const float* in, uint32_t N, uint64_t F, int8_t* out)
{
    for (uint64_t f = 0; f < F; ++f)
        for (unsigned i = 0; i < N; ++i) {
            const float x = in[f * N + i];
            out[f * N + i] = N >= 32 ? f2c_large(x) : N >= 8 ? f2c_vec(x) : f2c_scalar(x);
        }
}

/* ------------------------------------------------------------------ */
/* shared: frozen split, info packing, re-encode                        */
/* ------------------------------------------------------------------ */
static void csplit(const uint32_t* f, unsigned nf, unsigned half, uint32_t* l, unsigned* nl, uint32_t* r,
                   unsigned* nr)
{
    *nl = *nr = 0;
    for (unsigned i = 0; i < nf; ++i) {
        if (f[i] < half) l[(*nl)++] = f[i];
        else r[(*nr)++] = f[i] - half;
    }
}

/* CharContainer::getPackedInformationBits (bitcontainer.cpp:536-564) on the sign bits, or
 * (non-systematic) Encoder::setCharCodeword + ButterflyFipPacked::encode with
 * setSystematic(false) + getInformation (fastssc_fip_char.cpp:616-631). */
static void char_info(const int8_t* cw, unsigned N, const uint8_t* isf, int systematic, uint8_t* x, uint8_t* out)
{
    for (unsigned i = 0; i < N; ++i) x[i] = (uint8_t)((uint8_t)cw[i] >> 7);
    if (!systematic)
        for (unsigned B = 1; B < N; B <<= 1)
            for (unsigned j = 0; j < N; j += 2 * B)
                for (unsigned i = j; i < j + B; ++i) x[i] ^= x[i + B];
    unsigned K = 0;
    for (unsigned i = 0; i < N; ++i) K += !isf[i];
    memset(out, 0, (K + 7) / 8);
    unsigned j = 0;
    for (unsigned i = 0; i < N; ++i) {
        if (isf[i]) continue;
        if (x[i]) out[j / 8] |= (uint8_t)(0x80u >> (j % 8));
        ++j;
    }
}

static int cargs(unsigned N, const uint32_t* frozen, unsigned nf)
{
    if (N < 8 || (N & (N - 1)) || nf > N) return -1;
    for (unsigned i = 0; i < nf; ++i) {
        if (frozen[i] >= N) return -1;
        if (i && frozen[i] <= frozen[i - 1]) return -1;
    }
    return 0;
}

static unsigned vbytes(unsigned n) { return n < BV ? BV : n; } /* nBit2cvecCount(n) * 32 */

/* ================================================================== */
/* FastSscFipChar                src/polarcode/decoding/fastssc_fip_char.cpp */
/* ================================================================== */
enum {
    FC_R0 = 0,  /* RateZeroDecoder            :202-208 */
    FC_R1,      /* RateOneDecoder             :210-215 */
    FC_REP,     /* RepetitionDecoder (n>32)   :225-241 */
    FC_REPS,    /* ShortRepetitionDecoder     :265-272 */
    FC_SPC,     /* SpcDecoder (n>32)          :274-303 */
    FC_SPCS,    /* ShortSpcDecoder            :305-319 */
    FC_DREP,    /* DoubleRepetitionDecoder    :249-263 (n >= 32, no frozen-set check) */
    FC_ZONES,   /* ShortZeroOneDecoder        :390-399 */
    FC_ZSPCS,   /* ShortZeroSpcDecoder        :361-388 */
    FC_ZSPC,    /* ZeroSpcDecoder (n>32)      :321-359 */
    FC_RONE,    /* ROneNode                   :427-449 */
    FC_RONES,   /* ShortROneNode              :451-474 */
    FC_ZEROR,   /* ZeroRNode                  :476-483 */
    FC_ZERORS,  /* ShortZeroRNode             :485-492 */
    FC_RATER,   /* RateRNode                  :401-412 */
    FC_RATERS,  /* ShortRateRNode             :414-425 */
    FC_NTYPES
};

typedef struct fc_node {
    int type;
    unsigned n;
    struct fc_node *l, *r;
    int8_t* child; /* ChildLlr, vbytes(n/2) */
    int8_t* lb;    /* ShortNode LeftBits / ShortRateR LeftBits, 32 B */
    int8_t* rb;    /* RightBits, 32 B */
} fc_node;

static void fc_free(fc_node* x)
{
    if (!x) return;
    fc_free(x->l);
    fc_free(x->r);
    free(x->child);
    free(x->lb);
    free(x->rb);
    free(x);
}

/* FastSscFip::createDecoder, fastssc_fip_char.cpp:496-580 */
static fc_node* fc_create(const uint32_t* f, unsigned nf, unsigned n)
{
    fc_node* x = (fc_node*)calloc(1, sizeof(fc_node));
    x->n = n;
    x->lb = (int8_t*)calloc(BV, 1);
    x->rb = (int8_t*)calloc(BV, 1);
    if (nf == n) { x->type = FC_R0; return x; }
    if (nf == 0) { x->type = FC_R1; return x; }
    if (nf == n - 1) { x->type = n <= BV ? FC_REPS : FC_REP; return x; }
    if (nf == 1) { x->type = n <= BV ? FC_SPCS : FC_SPC; return x; }
    if (nf == n - 2 && n >= BV) { x->type = FC_DREP; return x; }
    const unsigned h = n / 2;
    uint32_t* lf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    uint32_t* rf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    unsigned nl, nr;
    csplit(f, nf, h, lf, &nl, rf, &nr);
    int leafonly = 0;
    if (n <= BV) {
        if (nl == h && nr == 0) { x->type = FC_ZONES; leafonly = 1; }
        else if (nl == h && nr == 1) { x->type = FC_ZSPCS; leafonly = 1; }
        else if (nr == 0) x->type = FC_RONES;
        else if (nl == h) x->type = FC_ZERORS;
        else x->type = FC_RATERS;
    } else {
        if (nl == h && nr == 1) { x->type = FC_ZSPC; leafonly = 1; }
        else if (nr == 0) x->type = FC_RONE;
        else if (nl == h) x->type = FC_ZEROR;
        else x->type = FC_RATER;
    }
    if (!leafonly) {
        x->l = fc_create(lf, nl, h);
        x->r = fc_create(rf, nr, h);
        x->child = (int8_t*)calloc(vbytes(h), 1);
    }
    free(lf);
    free(rf);
    return x;
}

/* F_function / G_function / G_function_0R(Short), fip_char.h:67-131 */
static void fc_F(const int8_t* in, int8_t* out, unsigned h)
{
    if (h < BV) {
        int8_t r[BV];
        vshift(in, r, h);
        for (unsigned i = 0; i < BV; ++i) out[i] = fip_f(in[i], r[i]);
    } else {
        for (unsigned i = 0; i < h; ++i) out[i] = fip_f(in[i], in[i + h]);
    }
}
static void fc_G(const int8_t* in, int8_t* out, const int8_t* bits, unsigned h)
{
    if (h < BV) {
        int8_t r[BV];
        vshift(in, r, h);
        for (unsigned i = 0; i < BV; ++i) out[i] = fip_g(in[i], r[i], bits[i]);
    } else {
        for (unsigned i = 0; i < h; ++i) out[i] = fip_g(in[i], in[i + h], bits[i]);
    }
}
static void fc_G0(const int8_t* in, int8_t* out, unsigned h)
{
    if (h < BV) {
        int8_t r[BV];
        vshift(in, r, h);
        for (unsigned i = 0; i < BV; ++i) out[i] = adds8(in[i], r[i]);
    } else {
        for (unsigned i = 0; i < h; ++i) out[i] = adds8(in[i], in[i + h]);
    }
}
/* CombineBitsShort, fip_char.h:180-201 (zeroes lanes >= h of L and R in place) */
static void combine_short(int8_t* L, int8_t* R, int8_t* out, unsigned h)
{
    int8_t lv[BV], rv[BV], rs[BV];
    memset(L + h, 0, BV - h);
    memset(R + h, 0, BV - h);
    for (unsigned i = 0; i < BV; ++i) {
        lv[i] = max8(L[i], -127);
        rv[i] = max8(R[i], -127);
    }
    vbackshift(rv, rs, h);
    for (unsigned i = 0; i < BV; ++i) out[i] = (int8_t)((lv[i] ^ rv[i]) | rs[i]);
}

/* SpcDecoder / ZeroSpcDecoder minimum search (fastssc_fip_char.cpp:287-297, 336-350):
 * per vector minpos, taken only if strictly below the running minimum (init 127),
 * search stops once a zero was found. */
static void fc_decode(fc_node* x, int8_t* in, int8_t* out)
{
    const unsigned n = x->n, h = n / 2;
    switch (x->type) {
    case FC_R0:
        memset(out, 127, vbytes(n));
        return;
    case FC_R1:
        memcpy(out, in, vbytes(n));
        return;
    case FC_REP: {
        int8_t acc[BV];
        memset(acc, 0, BV);
        for (unsigned v = 0; v < n / BV; ++v)
            for (unsigned i = 0; i < BV; ++i) acc[i] = adds8(acc[i], in[v * BV + i]);
        memset(out, reduce_adds(acc), n);
        return;
    }
    case FC_REPS:
        if (n < BV) memset(in + n, 0, BV - n); /* RepetitionPrepare */
        memset(out, reduce_adds(in), BV);
        return;
    case FC_DREP: {
        int8_t acc[BV], r[BV];
        memset(acc, 0, BV);
        for (unsigned v = 0; v < n / BV; ++v)
            for (unsigned i = 0; i < BV; ++i) acc[i] = adds8(acc[i], in[v * BV + i]);
        half_reduce_adds(acc, r);
        for (unsigned v = 0; v < n / BV; ++v) memcpy(out + v * BV, r, BV);
        return;
    }
    case FC_SPC: {
        unsigned mi = 0;
        int8_t ma = 127, t;
        uint8_t par = 0;
        for (unsigned v = 0; v < n / BV; ++v) {
            const int8_t* vi = in + v * BV;
            memcpy(out + v * BV, vi, BV);
            par ^= reduce_xor(vi);
            if (ma > 0) {
                int8_t a[BV];
                for (unsigned i = 0; i < BV; ++i) a[i] = abs8(vi[i]);
                const unsigned vm = minpos_epu8(a, &t);
                if (t < ma) { mi = vm + v * BV; ma = t; }
            }
        }
        if (par & 0x80) out[mi] = neg8(out[mi]);
        return;
    }
    case FC_SPCS: {
        if (n < BV) memset(in + n, 127, BV - n); /* SpcPrepare */
        memcpy(out, in, BV);
        if (reduce_xor(in) & 0x80) {
            int8_t a[BV];
            for (unsigned i = 0; i < BV; ++i) a[i] = abs8(in[i]);
            const unsigned vm = minpos_epu8(a, NULL);
            out[vm] = neg8(out[vm]);
        }
        return;
    }
    case FC_ZSPC: {
        unsigned mi = 0;
        int8_t ma = 127, t;
        uint8_t par = 0;
        for (unsigned v = 0; v < h / BV; ++v) {
            int8_t l[BV];
            for (unsigned i = 0; i < BV; ++i) l[i] = adds8(in[v * BV + i], in[h + v * BV + i]);
            memcpy(out + v * BV, l, BV);
            memcpy(out + h + v * BV, l, BV);
            par ^= reduce_xor(l);
            if (ma > 0) {
                int8_t a[BV];
                for (unsigned i = 0; i < BV; ++i) a[i] = abs8(l[i]);
                const unsigned vm = minpos_epu8(a, &t);
                if (t < ma) { mi = vm + v * BV; ma = t; }
            }
        }
        if (par & 0x80) {
            out[mi] = neg8(out[mi]);
            out[mi + h] = neg8(out[mi + h]);
        }
        return;
    }
    case FC_ZSPCS: {
        int8_t r[BV], l[BV];
        vshift(in, r, h);
        for (unsigned i = 0; i < BV; ++i) l[i] = adds8(in[i], r[i]);
        memset(l + h, 127, BV - h);
        if (reduce_xor(l) & 0x80) {
            int8_t a[BV];
            for (unsigned i = 0; i < BV; ++i) a[i] = abs8(l[i]);
            const unsigned vm = minpos_epu8(a, NULL);
            l[vm] = neg8(l[vm]);
        }
        memcpy(out, l, h);
        memcpy(out + h, l, h);
        return;
    }
    case FC_ZONES: {
        int8_t sl[BV], sr[BV];
        fc_G0(in, sl, h);
        vbackshift(sl, sr, h);
        memset(sl + h, 0, BV - h);
        for (unsigned i = 0; i < BV; ++i) out[i] = (int8_t)(sl[i] | sr[i]);
        return;
    }
    case FC_RATER:
        fc_F(in, x->child, h);
        fc_decode(x->l, x->child, out);
        fc_G(in, x->child, out, h);
        fc_decode(x->r, x->child, out + h);
        for (unsigned i = 0; i < h; ++i) out[i] ^= out[i + h]; /* CombineInPlace */
        return;
    case FC_RATERS:
        fc_F(in, x->child, h);
        fc_decode(x->l, x->child, x->lb);
        fc_G(in, x->child, x->lb, h);
        fc_decode(x->r, x->child, x->rb);
        combine_short(x->lb, x->rb, out, h);
        return;
    case FC_RONE:
        fc_F(in, x->child, h);
        fc_decode(x->l, x->child, out);
        for (unsigned i = 0; i < h; ++i) { /* simplifiedRightRateOneDecode :436-449 */
            const int8_t o = fip_g(in[i], in[i + h], out[i]);
            out[i] = (int8_t)(out[i] ^ o);
            out[i + h] = o;
        }
        return;
    case FC_RONES: {
        fc_F(in, x->child, h);
        fc_decode(x->l, x->child, out);
        int8_t b[BV], lr[BV], br[BV];
        memcpy(b, out, BV);
        fc_G(in, lr, out, h); /* simplifiedRightRateOneDecodeShort :460-474 */
        vbackshift(lr, br, h);
        for (unsigned i = 0; i < BV; ++i) b[i] = (int8_t)(b[i] ^ lr[i]);
        memset(b + h, 0, h);
        for (unsigned i = 0; i < BV; ++i) out[i] = (int8_t)(b[i] | br[i]);
        return;
    }
    case FC_ZEROR:
        fc_G0(in, x->child, h);
        fc_decode(x->r, x->child, out + h);
        memcpy(out, out + h, h); /* Combine_0R */
        return;
    case FC_ZERORS:
        fc_G0(in, x->child, h);
        fc_decode(x->r, x->child, x->rb);
        memcpy(out, x->rb, h); /* Combine_0RShort */
        memcpy(out + h, x->rb, h);
        return;
    default:
        return;
    }
}

static int fc_walk(const fc_node* x, int32_t* t, int32_t* s, int k, int maxn)
{
    if (!x) return k;
    if (k < maxn) { t[k] = x->type; s[k] = (int32_t)x->n; }
    k++;
    k = fc_walk(x->l, t, s, k, maxn);
    return fc_walk(x->r, t, s, k, maxn);
}

/* Node-type census (pre-order) of the FastSscFip tree; returns the node count. */
int orc_scc_tree(uint32_t N, const uint32_t* frozen, uint32_t nf, int32_t* types, int32_t* sizes, int maxn)
{
    if (cargs(N, frozen, nf)) return -1;
    fc_node* root = fc_create(frozen, nf, N);
    int k = fc_walk(root, types, sizes, 0, maxn);
    fc_free(root);
    return k;
}

/* Batched FastSscFipChar decode of int8 LLRs (decode_vector(const char*), decoder.cpp:169-181).
 * info F x ceil(K/8); ok F (nullable); softcw F x N int8 (nullable) = getSoftCodeword. */
int orc_scc_decode(uint32_t N, const uint32_t* frozen, uint32_t nf, int systematic, int crc, const int8_t* llr,
                   uint64_t F, uint8_t* info, uint8_t* ok, int8_t* softcw)
{
    if (cargs(N, frozen, nf)) return -1;
    fc_node* root = fc_create(frozen, nf, N);
    const unsigned kb = (N - nf + 7) / 8;
    uint8_t* isf = (uint8_t*)calloc(N, 1);
    for (unsigned i = 0; i < nf; ++i) isf[frozen[i]] = 1;
    int8_t* in = (int8_t*)calloc(vbytes(N), 1);
    int8_t* out = (int8_t*)calloc(vbytes(N), 1);
    uint8_t* x = (uint8_t*)malloc(N);
    for (uint64_t f = 0; f < F; ++f) {
        memcpy(in, llr + f * N, N);
        fc_decode(root, in, out);
        uint8_t* o = info + f * kb;
        char_info(out, N, isf, systematic, x, o);
        if (ok) ok[f] = (uint8_t)(orc_crc(crc, 0, o, (int)kb) > 0);
        if (softcw) memcpy(softcw + f * N, out, N);
    }
    free(in); free(out); free(x); free(isf);
    fc_free(root);
    return 0;
}

/* ================================================================== */
/* SclFipChar                    src/polarcode/decoding/scl_fip_char.cpp */
/* ================================================================== */
enum { FL_R0 = 0, FL_R1, FL_REP, FL_SPC, FL_RATER };

typedef struct fl_node {
    int type;
    unsigned n, s;
    struct fl_node *l, *r;
} fl_node;

static void fl_free(fl_node* x)
{
    if (!x) return;
    fl_free(x->l);
    fl_free(x->r);
    free(x);
}

/* SclFip::createDecoder, scl_fip_char.cpp:729-752 (ShortRateRNode = RateRNode on signs) */
static fl_node* fl_create(const uint32_t* f, unsigned nf, unsigned n)
{
    fl_node* x = (fl_node*)calloc(1, sizeof(fl_node));
    x->n = n;
    x->s = (unsigned)__builtin_ctz(n);
    if (nf == n) { x->type = FL_R0; return x; }
    if (nf == 0) { x->type = FL_R1; return x; }
    if (nf == n - 1) { x->type = FL_REP; return x; }
    if (nf == 1) { x->type = FL_SPC; return x; }
    x->type = FL_RATER;
    const unsigned h = n / 2;
    uint32_t* lf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    uint32_t* rf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    unsigned nl, nr;
    csplit(f, nf, h, lf, &nl, rf, &nr);
    x->l = fl_create(lf, nl, h);
    x->r = fl_create(rf, nr, h);
    free(lf);
    free(rf);
    return x;
}

typedef struct {
    unsigned L, S, P, stride, N;
    int cur;
    int8_t *llr[2], *bit[2], *lbit[2]; /* [L][S][stride] */
    long long metric[2][64];
    long long cm[8 * 64];
    unsigned cidx[8 * 64];
    unsigned nflip[8 * 64], flip[8 * 64][4];
    int8_t res[2 * 64];
    unsigned* widx;
    int8_t* tmp;
} fl_state;

#define FLP(st, arr, w, p, s) ((st)->arr[w] + ((size_t)(p) * (st)->S + (s)) * (st)->stride)

/* simplePartialSortDescending<unsigned,long> (arrayfuncs.h:161-183) */
static void sort_desc_ll(unsigned* idx, long long* v, unsigned n, unsigned size)
{
    for (unsigned i = 0; i < size; ++i) idx[i] = i;
    const unsigned lim = size - 1 < n ? size - 1 : n;
    for (unsigned i = 0; i < lim; ++i) {
        unsigned b = i;
        for (unsigned j = i + 1; j < size; ++j)
            if (v[j] > v[b]) b = j;
        long long tv = v[i]; v[i] = v[b]; v[b] = tv;
        unsigned ti = idx[i]; idx[i] = idx[b]; idx[b] = ti;
    }
}
/* findWeakLlrs<unsigned,char> (arrayfuncs.h:209-231) */
static void find_weak_c(unsigned* idx, int8_t* v, unsigned size, unsigned n)
{
    for (unsigned i = 0; i < size; ++i) idx[i] = i;
    const unsigned lim = size - 1 < n ? size - 1 : n;
    for (unsigned i = 0; i < lim; ++i) {
        unsigned b = i;
        for (unsigned j = i + 1; j < size; ++j)
            if (v[j] < v[b]) b = j;
        int8_t tv = v[i]; v[i] = v[b]; v[b] = tv;
        unsigned ti = idx[i]; idx[i] = idx[b]; idx[b] = ti;
    }
}

static void fl_dup(fl_state* st, unsigned dst, unsigned src, unsigned s)
{
    const int c = st->cur, x = 1 - c;
    for (unsigned k = s; k < st->S; ++k) {
        memcpy(FLP(st, llr, x, dst, k), FLP(st, llr, c, src, k), st->stride);
        memcpy(FLP(st, bit, x, dst, k), FLP(st, bit, c, src, k), st->stride);
        memcpy(FLP(st, lbit, x, dst, k), FLP(st, lbit, c, src, k), st->stride);
    }
}

/* sort, duplicatePath, metrics, NextBit = NextLlr (or Rep fill) + flips, switchToNext
 * (RateOneDecoder :472-505, RepetitionDecoder :562-580, SpcDecoder :697-726) */
static void fl_branch(fl_state* st, const fl_node* x, unsigned k)
{
    const unsigned P = st->P, size = k * P, vb = vbytes(x->n);
    const unsigned np = size < st->L ? size : st->L;
    sort_desc_ll(st->cidx, st->cm, np, size);
    for (unsigned p = 0; p < np; ++p) fl_dup(st, p, st->cidx[p] / k, x->s);
    st->cur = 1 - st->cur;
    st->P = np;
    for (unsigned p = 0; p < np; ++p) {
        const unsigned c = st->cidx[p];
        st->metric[st->cur][p] = st->cm[p];
        int8_t* b = FLP(st, bit, st->cur, p, x->s);
        if (x->type == FL_REP) {
            memset(b, st->res[c], vb);
        } else {
            memcpy(b, FLP(st, llr, st->cur, p, x->s), vb);
            for (unsigned i = 0; i < st->nflip[c]; ++i) b[st->flip[c][i]] = (int8_t)~b[st->flip[c][i]];
        }
    }
}

static void fl_leaf(fl_state* st, const fl_node* x)
{
    const unsigned n = x->n, s = x->s, P = st->P, vb = vbytes(n);
    const int c = st->cur;
    switch (x->type) {
    case FL_R0: /* RateZeroDecoder :387-421 */
        for (unsigned p = 0; p < P; ++p) {
            int8_t* v = FLP(st, llr, c, p, s);
            if (n < BV) memset(v + n, 0, BV - n);
            memset(FLP(st, bit, c, p, s), 127, vb);
            long long pun = 0;
            for (unsigned i = 0; i < vb; ++i) pun += v[i] < 0 ? v[i] : 0;
            st->metric[c][p] += pun;
        }
        return;
    case FL_R1: /* RateOneDecoder :423-470 */
        for (unsigned p = 0; p < P; ++p) {
            const long long m = st->metric[c][p];
            int8_t* v = FLP(st, llr, c, p, s);
            if (n < BV) memset(v + n, 127, BV - n);
            for (unsigned i = 0; i < vb; ++i) st->tmp[i] = abs8(max8(v[i], -127));
            find_weak_c(st->widx, st->tmp, n, 2);
            st->cm[4 * p] = m;
            st->cm[4 * p + 1] = m - st->tmp[0];
            if (n == 1) {
                st->cm[4 * p + 2] = -0x100000000000LL;
                st->cm[4 * p + 3] = -0x100000000000LL;
            } else {
                st->cm[4 * p + 2] = m - st->tmp[1];
                st->cm[4 * p + 3] = m - st->tmp[0] - st->tmp[1];
            }
            st->nflip[4 * p] = 0;
            st->nflip[4 * p + 1] = 1; st->flip[4 * p + 1][0] = st->widx[0];
            st->nflip[4 * p + 2] = 1; st->flip[4 * p + 2][0] = st->widx[1];
            st->nflip[4 * p + 3] = 2; st->flip[4 * p + 3][0] = st->widx[0]; st->flip[4 * p + 3][1] = st->widx[1];
        }
        fl_branch(st, x, 4);
        return;
    case FL_REP: /* RepetitionDecoder :508-580 */
        for (unsigned p = 0; p < P; ++p) {
            const long long m = st->metric[c][p];
            int8_t* v = FLP(st, llr, c, p, s);
            if (n < BV) memset(v + n, 0, BV - n);
            int8_t acc[BV];
            memset(acc, 0, BV);
            long long z = 0, o = 0;
            for (unsigned q = 0; q < vb / BV; ++q)
                for (unsigned i = 0; i < BV; ++i) {
                    const int8_t l = v[q * BV + i];
                    acc[i] = adds8(acc[i], l);
                    z += l < 0 ? l : 0;
                    o += l > 0 ? l : 0;
                }
            const int8_t r = max8(reduce_adds(acc), -127);
            st->res[2 * p] = r < 0 ? (int8_t)~r : r;
            st->res[2 * p + 1] = r < 0 ? r : (int8_t)~r;
            st->cm[2 * p] = m + z;
            st->cm[2 * p + 1] = m - o;
        }
        fl_branch(st, x, 2);
        return;
    case FL_SPC: /* SpcDecoder :583-726 */
        for (unsigned p = 0; p < P; ++p) {
            long long m = st->metric[c][p];
            int8_t* v = FLP(st, llr, c, p, s);
            if (n < BV) memset(v + n, 127, BV - n);
            uint8_t par = 0;
            for (unsigned i = 0; i < vb; ++i) {
                par ^= (uint8_t)v[i];
                st->tmp[i] = abs8(max8(v[i], -127));
            }
            find_weak_c(st->widx, st->tmp, n, 4);
            const long long T0 = st->tmp[0], T1 = st->tmp[1], T2 = st->tmp[2], T3 = st->tmp[3];
            const unsigned i0 = st->widx[0], i1 = st->widx[1], i2 = st->widx[2], i3 = st->widx[3];
            unsigned* nf = st->nflip + 8 * p;
            unsigned(*fl)[4] = st->flip + 8 * p;
            long long weakest = 0;
            if (par & 0x80) {
                m -= T0;
                nf[0] = 1; fl[0][0] = i0;
                nf[1] = nf[2] = nf[3] = 0;
                nf[4] = 1; fl[4][0] = i0;
                nf[5] = 1; fl[5][0] = i0;
                nf[6] = 1; fl[6][0] = i0;
                nf[7] = 0;
            } else {
                nf[0] = 0;
                nf[1] = 1; fl[1][0] = i0;
                nf[2] = 1; fl[2][0] = i0;
                nf[3] = 1; fl[3][0] = i0;
                nf[4] = nf[5] = nf[6] = 0;
                nf[7] = 1; fl[7][0] = i0;
                weakest = T0;
            }
            long long* cm = st->cm + 8 * p;
            cm[0] = m;
            cm[1] = m - weakest - T1;
            cm[2] = m - weakest - T2;
            cm[3] = m - weakest - T3;
            cm[4] = m - T1 - T2;
            cm[5] = m - T1 - T3;
            cm[6] = m - T2 - T3;
            cm[7] = m - weakest - T1 - T2 - T3;
            fl[1][nf[1]++] = i1;
            fl[2][nf[2]++] = i2;
            fl[3][nf[3]++] = i3;
            fl[4][nf[4]++] = i1; fl[4][nf[4]++] = i2;
            fl[5][nf[5]++] = i1; fl[5][nf[5]++] = i3;
            fl[6][nf[6]++] = i2; fl[6][nf[6]++] = i3;
            fl[7][nf[7]++] = i1; fl[7][nf[7]++] = i2; fl[7][nf[7]++] = i3;
        }
        fl_branch(st, x, 8);
        return;
    default:
        return;
    }
}

/* RateRNode::decode / ShortRateRNode::decode, scl_fip_char.cpp:315-385 */
static void fl_decode(fl_state* st, const fl_node* x)
{
    if (x->type != FL_RATER) {
        fl_leaf(st, x);
        return;
    }
    const unsigned cs = x->s - 1, h = x->n / 2;
    for (unsigned p = 0; p < st->P; ++p)
        fc_F(FLP(st, llr, st->cur, p, cs + 1), FLP(st, llr, st->cur, p, cs), h);
    fl_decode(st, x->l);
    for (unsigned p = 0; p < st->P; ++p) { /* prepareRightDecoding: swap Bit / LeftBit */
        int8_t* a = FLP(st, bit, st->cur, p, cs);
        int8_t* b = FLP(st, lbit, st->cur, p, cs);
        for (unsigned i = 0; i < st->stride; ++i) { int8_t t = a[i]; a[i] = b[i]; b[i] = t; }
    }
    for (unsigned p = 0; p < st->P; ++p)
        fc_G(FLP(st, llr, st->cur, p, cs + 1), FLP(st, llr, st->cur, p, cs), FLP(st, lbit, st->cur, p, cs), h);
    fl_decode(st, x->r);
    for (unsigned p = 0; p < st->P; ++p) {
        int8_t* L = FLP(st, lbit, st->cur, p, cs);
        int8_t* R = FLP(st, bit, st->cur, p, cs);
        int8_t* O = FLP(st, bit, st->cur, p, cs + 1);
        if (h >= BV) { /* CombineBits fip_char.h:165-178 */
            for (unsigned i = 0; i < h; ++i) {
                O[i] = (int8_t)(L[i] ^ R[i]);
                O[i + h] = R[i];
            }
        } else {
            combine_short(L, R, O, h);
        }
    }
}

int orc_sclc_tree(uint32_t N, const uint32_t* frozen, uint32_t nf, int32_t* types, int32_t* sizes, int maxn);
static int fl_walk(const fl_node* x, int32_t* t, int32_t* s, int k, int maxn)
{
    if (!x) return k;
    if (k < maxn) { t[k] = x->type; s[k] = (int32_t)x->n; }
    k++;
    k = fl_walk(x->l, t, s, k, maxn);
    return fl_walk(x->r, t, s, k, maxn);
}
int orc_sclc_tree(uint32_t N, const uint32_t* frozen, uint32_t nf, int32_t* types, int32_t* sizes, int maxn)
{
    if (cargs(N, frozen, nf)) return -1;
    fl_node* root = fl_create(frozen, nf, N);
    int k = fl_walk(root, types, sizes, 0, maxn);
    fl_free(root);
    return k;
}

/* Batched SclFipChar decode of int8 LLRs.  carry != 0: path 0's metric is carried from
 * frame to frame (PathList::clear / setFirstPath never reset mMetric,
 * scl_fip_char.cpp:49-53, 100-107) -- an offset of every integer metric of the frame, so
 * it changes reported metrics but no decision.  metrics F x L (int64, nullable),
 * pathcount F (nullable), pathbits F x L x N/8 (nullable). */
int orc_sclc_decode(uint32_t N, uint32_t L, const uint32_t* frozen, uint32_t nf, int systematic, int crc, int carry,
                    const int8_t* llr, uint64_t F, uint8_t* info, uint8_t* ok, int64_t* metrics,
                    uint32_t* pathcount, uint8_t* pathbits)
{
    if (cargs(N, frozen, nf) || L < 1 || L > 64) return -1;
    fl_node* root = fl_create(frozen, nf, N);
    fl_state* st = (fl_state*)calloc(1, sizeof(fl_state));
    st->L = L;
    st->N = N;
    st->S = (unsigned)__builtin_ctz(N) + 1;
    st->stride = vbytes(N);
    st->widx = (unsigned*)calloc(N + BV, sizeof(unsigned));
    st->tmp = (int8_t*)calloc(N + BV, 1);
    const size_t tot = (size_t)L * st->S * st->stride;
    for (int w = 0; w < 2; ++w) {
        st->llr[w] = (int8_t*)calloc(tot, 1);
        st->bit[w] = (int8_t*)calloc(tot, 1);
        st->lbit[w] = (int8_t*)calloc(tot, 1);
    }
    const unsigned kb = (N - nf + 7) / 8, top = st->S - 1;
    uint8_t* isf = (uint8_t*)calloc(N, 1);
    for (unsigned i = 0; i < nf; ++i) isf[frozen[i]] = 1;
    uint8_t* x = (uint8_t*)malloc(N);
    uint8_t* o = (uint8_t*)malloc(kb + 8);
    long long carried = 0;
    for (uint64_t f = 0; f < F; ++f) {
        st->cur = 0;
        st->P = 1;
        st->metric[0][0] = carry ? carried : 0;
        memcpy(FLP(st, llr, 0, 0, top), llr + f * N, N);
        fl_decode(st, root);
        const unsigned P = st->P;
        int found = 0; /* extractBestPath :816-856 */
        for (unsigned p = 0; p < P && !found; ++p) {
            char_info(FLP(st, bit, st->cur, p, top), N, isf, systematic, x, o);
            if (orc_crc(crc, 0, o, (int)kb) > 0) found = 1;
        }
        if (!found) char_info(FLP(st, bit, st->cur, 0, top), N, isf, systematic, x, o);
        memcpy(info + f * kb, o, kb);
        if (ok) ok[f] = (uint8_t)found;
        carried = st->metric[st->cur][0];
        if (pathcount) pathcount[f] = P;
        for (unsigned p = 0; p < L; ++p) {
            if (metrics) metrics[f * L + p] = p < P ? st->metric[st->cur][p] : 0;
            if (pathbits) {
                uint8_t* pb = pathbits + (f * L + p) * (N / 8);
                memset(pb, 0, N / 8);
                if (p < P) {
                    const int8_t* b = FLP(st, bit, st->cur, p, top);
                    for (unsigned i = 0; i < N; ++i)
                        if ((uint8_t)b[i] & 0x80u) pb[i / 8] |= (uint8_t)(0x80u >> (i % 8));
                }
            }
        }
    }
    for (int w = 0; w < 2; ++w) { free(st->llr[w]); free(st->bit[w]); free(st->lbit[w]); }
    free(st->widx); free(st->tmp);
    free(st); free(isf); free(x); free(o);
    fl_free(root);
    return 0;
}

/* ------------------------------------------------------------------ */
/* element kernels, exported for the reference's known-answer tests    */
/* (test/polarcode/decodingtest.cpp, testGeneralDecodingFunctionsAvx2) */
/* ------------------------------------------------------------------ */
/* in: 2h bytes (h >= 32: left half, right half; h < 32: one 32-byte vector) */
void orc_fip_f(const int8_t* in, int8_t* out, uint32_t h) { fc_F(in, out, h); }
void orc_fip_g(const int8_t* in, const int8_t* bits, int8_t* out, uint32_t h) { fc_G(in, out, bits, h); }
/* 32-byte L, R (modified in place as the reference does), 32-byte out */
void orc_fip_combine_short(int8_t* l, int8_t* r, int8_t* out, uint32_t h) { combine_short(l, r, out, h); }
