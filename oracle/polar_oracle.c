/*
 * polar_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, scalar restatement of the reference's float Fast-SSC ("SC") and
 * SCL decoders (david13pod/antPolarCodes, mounted read-only at /root/reference),
 * including every lane-order / sign-of-zero / tie quirk the AVX2 code has, so
 * that it produces bit-identical outputs.  It is the CHECKER for the HIP path:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it
 * (oracle/liboracle.so via ctypes).  The product (antpolarcodes_amd/) never
 * links, loads or falls back to it.
 *
 * Pinning: tests/test_oracle.py checks this file against fixtures produced by
 * the reference itself (oracle/_ref/libpolarref.so, built from the reference
 * sources by oracle/Makefile; fixtures committed under tests/golden/ by
 * tests/golden/make_golden.py) and, when oracle/_ref is present, against the
 * reference directly on fresh random inputs.
 *
 * All citations: path:line relative to /root/reference.
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* float bit helpers (the reference works on IEEE bit patterns)        */
/* ------------------------------------------------------------------ */
typedef union {
    float f;
    uint32_t u;
} fu_t;

static inline uint32_t fb(float x) { fu_t v; v.f = x; return v.u; }
static inline float bf(uint32_t u) { fu_t v; v.u = u; return v.f; }
static inline float fxor(float a, float b) { return bf(fb(a) ^ fb(b)); }
static inline float fabs_(float a) { return bf(fb(a) & 0x7fffffffu); }
static inline float fsign(float a) { return bf(fb(a) & 0x80000000u); }
/* _mm256_min_ps / _mm256_max_ps: second operand on ties and NaN */
static inline float minps(float a, float b) { return a < b ? a : b; }
static inline float maxps(float a, float b) { return a > b ? a : b; }

/* F: sign(a)^sign(b) OR'ed onto min(|a|,|b|)   include/polarcode/decoding/avx_float.h:55-63 */
static inline float polar_f(float a, float b)
{
    return bf(((fb(a) ^ fb(b)) & 0x80000000u) | fb(minps(fabs_(a), fabs_(b))));
}
/* G: (a XOR signbit(bit)) + b                   avx_float.h:71-81 */
static inline float polar_g(float a, float b, float bit) { return fxor(a, fsign(bit)) + b; }

/* reduce_add_ps: x0+x1+...+x7 left to right      include/polarcode/avxconvenience.h:256-272 */
static inline float reduce_add8(const float* x)
{
    return x[0] + x[1] + x[2] + x[3] + x[4] + x[5] + x[6] + x[7];
}

/* 8 lane partial sums, each lane starting from +0.0 (_mm256_setzero_ps), chunks of 8
 * in ascending order; blocks shorter than 8 are padded with `pad` first
 * (RepetitionPrepare / SpcPrepare, avx_float.h:238-250). */
static void lane_sums(const float* in, unsigned n, float pad, float s[8])
{
    for (unsigned j = 0; j < 8; ++j)
        s[j] = 0.0f;
    if (n < 8) {
        for (unsigned j = 0; j < 8; ++j)
            s[j] = s[j] + (j < n ? in[j] : pad);
        return;
    }
    for (unsigned i = 0; i < n; i += 8)
        for (unsigned j = 0; j < 8; ++j)
            s[j] = s[j] + in[i + j];
}

/* 4-lane SPC of _mm256_spc_right4_ps (avx_float.h:289-302): every lane whose |v|
 * equals the minimum gets its sign flipped when the XOR of the 4 signs is 1. */
static void spc4(const float v[4], float out[4])
{
    float a[4], m;
    for (int k = 0; k < 4; ++k)
        a[k] = fabs_(v[k]);
    /* min network: lanes {k, k^2} then {k, k^1} */
    float t0 = minps(a[0], a[2]), t1 = minps(a[1], a[3]);
    m = minps(t0, t1);
    uint32_t par = (fb(v[0]) ^ fb(v[1]) ^ fb(v[2]) ^ fb(v[3])) & 0x80000000u;
    for (int k = 0; k < 4; ++k)
        out[k] = (a[k] == m) ? bf(fb(v[k]) ^ par) : v[k];
}

/* ------------------------------------------------------------------ */
/* frozen-set splitting      src/polarcode/polarcode.cpp:14-34         */
/* ------------------------------------------------------------------ */
static void split_frozen(const uint32_t* f,
                         unsigned nf,
                         unsigned half,
                         uint32_t* l,
                         unsigned* nl,
                         uint32_t* r,
                         unsigned* nr)
{
    *nl = *nr = 0;
    for (unsigned i = 0; i < nf; ++i) {
        if (f[i] < half)
            l[(*nl)++] = f[i];
        else
            r[(*nr)++] = f[i] - half;
    }
}

/* ================================================================== */
/* Fast-SSC (FastSscAvxFloat)   src/polarcode/decoding/fastssc_avx_float.cpp */
/* ================================================================== */
enum {
    SC_R0 = 0,     /* RateZeroDecoder                 :247            */
    SC_R1,         /* RateOneDecoder                  :257-263        */
    SC_REP,        /* RepetitionDecoder               :273-287        */
    SC_SPC,        /* SpcDecoder                      :342-373        */
    SC_DREP,       /* DoubleRepetitionDecoder         :303-332        */
    SC_DSPC,       /* DoubleSpcDecoder (n>=16)        :425-466        */
    SC_DSPC8,      /* DoubleSpcDecoderShort8          :473-488        */
    SC_TREP,       /* TripleRepetitionDecoder         :572-589        */
    SC_TYPE5,      /* TypeFiveDecoder                 :762-792        */
    SC_REPR1_8,    /* RepetitionRateOneDecoderShort8  :718-739        */
    SC_ZSPC8,      /* ZeroSpcDecoderShort8            :556-565        */
    SC_ZSPC,       /* ZeroSpcDecoder (n>8)            :503-546        */
    SC_RATER,      /* RateRNode / ShortRateRNode      :148-185        */
    SC_RONE,       /* ROneNode                        :198-219        */
    SC_ZEROR,      /* ZeroRNode                       :232-237        */
    SC_NTYPES
};

typedef struct sc_node {
    int type;
    unsigned n;
    struct sc_node *l, *r;
} sc_node;

static void sc_free(sc_node* x)
{
    if (!x)
        return;
    sc_free(x->l);
    sc_free(x->r);
    free(x);
}

/* createDecoder, fastssc_avx_float.cpp:797-896.  Returns NULL and sets *err = -2 on
 * the std::invalid_argument cases (:821-825, :839-843). */
static sc_node* sc_create(const uint32_t* f, unsigned nf, unsigned n, int* err)
{
    if (*err)
        return NULL;
    sc_node* x = (sc_node*)calloc(1, sizeof(sc_node));
    x->n = n;
    if (nf == n) { x->type = SC_R0; return x; }
    if (nf == 0) { x->type = SC_R1; return x; }
    if (nf == n - 1) { x->type = SC_REP; return x; }
    if (nf == 1) { x->type = SC_SPC; return x; }
    if (nf == n - 2) {
        for (unsigned i = 0; i < nf; ++i)
            if (f[i] != i) { *err = -2; free(x); return NULL; }
        if (n < 4) { *err = -2; free(x); return NULL; } /* :295-298 */
        x->type = SC_DREP;
        return x;
    }
    if (nf == 2 && f[0] == 0 && f[1] == 1) {
        x->type = (n == 8) ? SC_DSPC8 : SC_DSPC;
        return x;
    }
    if (nf == n - 3 && n > 8 && f[nf - 1] == n - 4) {
        for (unsigned i = 0; i < nf; ++i)
            if (f[i] != i) { *err = -2; free(x); return NULL; }
        x->type = SC_TREP;
        return x;
    }
    if (nf == n - 4 && f[nf - 1] == n - 4 && f[nf - 2] == n - 6) {
        x->type = SC_TYPE5;
        return x;
    }
    if (n == 8 && nf == 3 && f[0] == 0 && f[1] == 1 && f[2] == 2) {
        x->type = SC_REPR1_8;
        return x;
    }
    if (n == 8 && nf == 5 && f[nf - 1] == n - 4 && f[nf - 2] == n - 5) {
        x->type = SC_ZSPC8;
        return x;
    }
    /* (n == 8 here prints a WARNING in the reference, :864-870) */
    unsigned h = n / 2, nl, nr;
    uint32_t* lf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    uint32_t* rf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    split_frozen(f, nf, h, lf, &nl, rf, &nr);
    if (n <= 8) {
        x->type = SC_RATER; /* ShortRateRNode: same observable semantics */
        x->l = sc_create(lf, nl, h, err);
        x->r = sc_create(rf, nr, h, err);
    } else if (nl == h && nr == 1) {
        x->type = SC_ZSPC;
    } else if (nr == 0) {
        x->type = SC_RONE; /* right child is a dummy Node (NO_RIGHT) */
        x->l = sc_create(lf, nl, h, err);
    } else if (nl == h) {
        x->type = SC_ZEROR; /* left child is a dummy Node (NO_LEFT) */
        x->r = sc_create(rf, nr, h, err);
    } else {
        x->type = SC_RATER;
        x->l = sc_create(lf, nl, h, err);
        x->r = sc_create(rf, nr, h, err);
    }
    free(lf);
    free(rf);
    if (*err) {
        sc_free(x);
        return NULL;
    }
    return x;
}

/* leaf decoders; `in` has n floats, `out` receives n floats */
static void sc_leaf(const sc_node* x, const float* in, float* out)
{
    const unsigned n = x->n;
    float s[8];
    switch (x->type) {
    case SC_R0:
        for (unsigned i = 0; i < n; ++i)
            out[i] = INFINITY;
        break;
    case SC_R1:
        memcpy(out, in, 4 * n);
        break;
    case SC_REP: {
        lane_sums(in, n, 0.0f, s);
        float S = reduce_add8(s);
        for (unsigned i = 0; i < n; ++i)
            out[i] = S;
        break;
    }
    case SC_DREP: {
        lane_sums(in, n, 0.0f, s);
        float ev, od;
        if (n >= 8) {
            /* permute2f128 then shuffle 0x4E  (:314-321) */
            ev = (s[0] + s[4]) + (s[2] + s[6]);
            od = (s[1] + s[5]) + (s[3] + s[7]);
        } else {
            ev = s[0] + s[2] + s[4] + s[6];
            od = s[1] + s[3] + s[5] + s[7];
        }
        for (unsigned i = 0; i < n; i += 2) {
            out[i] = ev;
            out[i + 1] = od;
        }
        break;
    }
    case SC_SPC: {
        /* parity over all (padded) lanes; argmin = lowest index of min |x| */
        uint32_t par = 0;
        unsigned m = 0;
        float mv = INFINITY;
        const unsigned nn = n < 8 ? 8 : n;
        for (unsigned i = 0; i < nn; ++i) {
            float v = i < n ? in[i] : INFINITY;
            par ^= fb(v);
            float a = fabs_(v);
            if (a < mv) { mv = a; m = i; }
        }
        memcpy(out, in, 4 * n);
        if (m < n)
            out[m] = bf(fb(out[m]) ^ (par & 0x80000000u));
        break;
    }
    case SC_DSPC: {
        /* per-lane running argmin, ties -> later chunk (:257-266, mask is GT) */
        float mv[8];
        unsigned mi[8];
        uint32_t par[8] = { 0 };
        for (int j = 0; j < 8; ++j) { mv[j] = 3.40282347e+38f; mi[j] = 0; }
        for (unsigned i = 0; i < n; i += 8)
            for (unsigned j = 0; j < 8; ++j) {
                float v = in[i + j];
                par[j] ^= fb(v);
                float a = fabs_(v);
                if (!(a > mv[j])) { mv[j] = a; mi[j] = i + j; }
            }
        float ce = minps(minps(mv[0], mv[4]), minps(mv[2], mv[6]));
        float co = minps(minps(mv[1], mv[5]), minps(mv[3], mv[7]));
        unsigned ei = 0, oi = 0;
        for (int j = 6; j >= 0; j -= 2) if (mv[j] == ce) ei = mi[j];
        for (int j = 7; j >= 1; j -= 2) if (mv[j] == co) oi = mi[j];
        uint32_t pe = (par[0] ^ par[2] ^ par[4] ^ par[6]) & 0x80000000u;
        uint32_t po = (par[1] ^ par[3] ^ par[5] ^ par[7]) & 0x80000000u;
        memcpy(out, in, 4 * n);
        out[ei] = bf(fb(out[ei]) ^ pe);
        out[oi] = bf(fb(out[oi]) ^ po);
        break;
    }
    case SC_DSPC8: {
        float a[8];
        for (int j = 0; j < 8; ++j) a[j] = fabs_(in[j]);
        float ce = minps(minps(a[0], a[4]), minps(a[2], a[6]));
        float co = minps(minps(a[1], a[5]), minps(a[3], a[7]));
        uint32_t pe = (fb(in[0]) ^ fb(in[2]) ^ fb(in[4]) ^ fb(in[6])) & 0x80000000u;
        uint32_t po = (fb(in[1]) ^ fb(in[3]) ^ fb(in[5]) ^ fb(in[7])) & 0x80000000u;
        for (int j = 0; j < 8; ++j) {
            int ev = (j % 2) == 0;
            int hit = a[j] == (ev ? ce : co);
            out[j] = hit ? bf(fb(in[j]) ^ (ev ? pe : po)) : in[j];
        }
        break;
    }
    case SC_ZSPC8: {
        float v[4], o[4];
        for (int k = 0; k < 4; ++k) v[k] = in[k] + in[k + 4];
        spc4(v, o);
        for (int k = 0; k < 4; ++k) { out[k] = o[k]; out[k + 4] = o[k]; }
        break;
    }
    case SC_TREP: {
        lane_sums(in, n, 0.0f, s);
        float v[4], o[4];
        for (int k = 0; k < 4; ++k) v[k] = s[k] + s[k + 4];
        spc4(v, o);
        for (unsigned i = 0; i < n; ++i) out[i] = o[i % 4];
        break;
    }
    case SC_TYPE5:
    case SC_REPR1_8: {
        float l[8];
        if (x->type == SC_TYPE5)
            lane_sums(in, n, 0.0f, l);
        else
            memcpy(l, in, 32);
        float r[4];
        for (int k = 0; k < 4; ++k) r[k] = polar_f(l[k], l[k + 4]);
        /* hadd(hadd(.)) -> (r0+r1)+(r2+r3) */
        float R = (r[0] + r[1]) + (r[2] + r[3]);
        float g[4], o[4];
        for (int k = 0; k < 4; ++k) g[k] = polar_g(l[k], l[k + 4], R);
        if (x->type == SC_TYPE5)
            spc4(g, o);
        else
            memcpy(o, g, 16);
        float res[8];
        for (int k = 0; k < 4; ++k) {
            res[k] = bf(((fb(R) ^ fb(o[k])) & 0x80000000u) ^ fb(1.0f));
            res[k + 4] = o[k];
        }
        for (unsigned i = 0; i < n; ++i) out[i] = res[i % 8];
        break;
    }
    case SC_ZSPC: {
        /* Q1: outputs the RIGHT half to both halves (:519-520) */
        const unsigned h = n / 2;
        uint32_t par = 0;
        unsigned m = 0;
        float mv = INFINITY;
        for (unsigned i = 0; i < h; ++i) {
            float llr = in[i] + in[h + i];
            out[i] = in[h + i];
            out[h + i] = in[h + i];
            par ^= fb(llr);
            float a = fabs_(llr);
            if (a < mv) { mv = a; m = i; }
        }
        par &= 0x80000000u;
        out[m] = bf(fb(out[m]) ^ par);
        out[m + h] = bf(fb(out[m + h]) ^ par);
        break;
    }
    default:
        break;
    }
}

static void sc_decode_node(const sc_node* x, const float* in, float* out, float* scratch)
{
    const unsigned n = x->n, h = n / 2;
    float* llr = scratch; /* h floats for the child, rest for deeper levels */
    switch (x->type) {
    case SC_RATER:
        for (unsigned i = 0; i < h; ++i) llr[i] = polar_f(in[i], in[h + i]);
        sc_decode_node(x->l, llr, out, scratch + h);
        for (unsigned i = 0; i < h; ++i) llr[i] = polar_g(in[i], in[h + i], out[i]);
        sc_decode_node(x->r, llr, out + h, scratch + h);
        for (unsigned i = 0; i < h; ++i) out[i] = fxor(out[i], out[h + i]);
        break;
    case SC_RONE:
        for (unsigned i = 0; i < h; ++i) llr[i] = polar_f(in[i], in[h + i]);
        sc_decode_node(x->l, llr, out, scratch + h);
        for (unsigned i = 0; i < h; ++i) {
            float bits = out[i];
            float r = fxor(in[i], fsign(bits)) + in[h + i];
            out[i] = fxor(bits, r);
            out[h + i] = r;
        }
        break;
    case SC_ZEROR:
        for (unsigned i = 0; i < h; ++i) llr[i] = in[i] + in[h + i];
        sc_decode_node(x->r, llr, out + h, scratch + h);
        for (unsigned i = 0; i < h; ++i) out[i] = out[h + i];
        break;
    default:
        sc_leaf(x, in, out);
    }
}

/* ------------------------------------------------------------------ */
/* info-bit packing, non-systematic re-encode, detectors               */
/* ------------------------------------------------------------------ */

/* FloatContainer::getPackedInformationBits, src/polarcode/bitcontainer.cpp:225-292:
 * j-th non-frozen position -> byte j/8, bit 7-(j%8). */
static void pack_info(const uint8_t* cwbits, unsigned N, const uint8_t* isfrozen, uint8_t* out)
{
    unsigned K = 0;
    for (unsigned i = 0; i < N; ++i) K += !isfrozen[i];
    memset(out, 0, (K + 7) / 8);
    unsigned j = 0;
    for (unsigned i = 0; i < N; ++i) {
        if (isfrozen[i]) continue;
        if (cwbits[i]) out[j / 8] |= (uint8_t)(0x80u >> (j % 8));
        ++j;
    }
}

/* ButterflyFipPacked::transform (butterfly_fip_packed.cpp:60-70, butterfly_fip.cpp:15-63):
 * for each stage s: x[i] ^= x[i + 2^s] for i with bit s clear. */
static void polar_transform(uint8_t* x, unsigned N)
{
    for (unsigned B = 1; B < N; B <<= 1)
        for (unsigned j = 0; j < N; j += 2 * B)
            for (unsigned i = j; i < j + B; ++i) x[i] ^= x[i + B];
}

static uint8_t g_crc8_table[256];
static int g_crc8_init = 0;

/* CRC8 poly 0x07, init 0, check = last byte    errordetection/crc8.cpp:18-57 */
static uint8_t crc8_gen(const uint8_t* d, int bytes)
{
    if (!g_crc8_init) {
        for (int i = 0; i < 256; ++i) {
            uint8_t c = (uint8_t)i;
            for (int j = 0; j < 8; ++j) c = (uint8_t)((c << 1) ^ ((c & 0x80) ? 0x07 : 0));
            g_crc8_table[i] = c;
        }
        g_crc8_init = 1;
    }
    uint8_t c = 0;
    for (int i = 0; i < bytes; ++i) c = g_crc8_table[c ^ d[i]];
    return c;
}

/* CRC-16/CCITT-FALSE (0x1021, init 0xFFFF), big-endian in the last 2 bytes
 * errordetection/crc16.cpp:21-43 via CRC++ CRC_16_CCITTFALSE (CRC.h) */
static uint16_t crc16_gen(const uint8_t* d, int bytes)
{
    uint16_t c = 0xFFFF;
    for (int i = 0; i < bytes; ++i) {
        c ^= (uint16_t)(d[i] << 8);
        for (int b = 0; b < 8; ++b) c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x1021 : (c << 1));
    }
    return c;
}

/* CRC-32C over little-endian 32-bit words, init 0, no final xor (_mm_crc32_u32)
 * errordetection/crc32.cpp:28-66 */
static uint32_t crc32c_gen(const uint8_t* d, int words)
{
    uint32_t c = 0;
    for (int w = 0; w < words; ++w) {
        uint32_t v = (uint32_t)d[4 * w] | ((uint32_t)d[4 * w + 1] << 8) |
                     ((uint32_t)d[4 * w + 2] << 16) | ((uint32_t)d[4 * w + 3] << 24);
        c ^= v;
        for (int b = 0; b < 32; ++b) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    }
    return c;
}

/* CRC-11 -- NOT in the reference (parity unpinned).  3GPP TS 38.212
 * §5.1 gCRC11(D) = D^11+D^10+D^9+D^5+1, zero init, computed over the message bit
 * stream (bytes MSB-first); the parity bits are the last 11 bits, MSB first.  Written
 * as the textbook polynomial long division of m(D)*D^11 (a different formulation
 * from the product's shift register, so the two check each other). */
static uint32_t crc11_div(const uint8_t* d, int nbits)
{
    /* long division over a bit array: r holds 12 bits, shift in message then 11 zeros */
    uint32_t r = 0;
    for (int i = 0; i < nbits + 11; ++i) {
        uint32_t b = i < nbits ? (uint32_t)((d[i / 8] >> (7 - i % 8)) & 1) : 0u;
        r = (r << 1) | b;
        if (r & 0x800u) r ^= 0xE21u; /* 1110 0010 0001 = D^11+D^10+D^9+D^5+1 */
    }
    return r & 0x7FFu;
}

/* crc: -1 -> CRC-8 (what makeDecoder installs, decoder.cpp:85), 0 -> Dummy (always ok) */
int orc_crc(int crc, int generate, uint8_t* data, int bytes)
{
    if (crc < 0) crc = 8;
    switch (crc) {
    case 0:
        return 1;
    case 8: {
        uint8_t c = crc8_gen(data, bytes - 1);
        if (generate) { data[bytes - 1] = c; return 0; }
        return c == data[bytes - 1];
    }
    case 16: {
        uint16_t c = crc16_gen(data, bytes - 2);
        if (generate) {
            data[bytes - 2] = (uint8_t)(c >> 8);
            data[bytes - 1] = (uint8_t)c;
            return 0;
        }
        return c == (uint16_t)((data[bytes - 2] << 8) | data[bytes - 1]);
    }
    case 11: {
        int nb = bytes * 8 - 11;
        uint32_t c = crc11_div(data, nb), t = 0;
        for (int k = 0; k < 11; ++k) {
            int i = nb + k;
            uint8_t m = (uint8_t)(0x80u >> (i % 8));
            if (generate) {
                if ((c >> (10 - k)) & 1u) data[i / 8] |= m; else data[i / 8] &= (uint8_t)~m;
            } else {
                t = (t << 1) | (uint32_t)((data[i / 8] & m) != 0);
            }
        }
        return generate ? 0 : (int)(c == t);
    }
    case 32: {
        int rw = (bytes >> 2) - 1;
        uint32_t c = crc32c_gen(data, rw);
        uint8_t* p = data + 4 * rw;
        if (generate) {
            p[0] = (uint8_t)c; p[1] = (uint8_t)(c >> 8);
            p[2] = (uint8_t)(c >> 16); p[3] = (uint8_t)(c >> 24);
            return 0;
        }
        uint32_t s = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                     ((uint32_t)p[3] << 24);
        return c == s;
    }
    default:
        return -1;
    }
}

static void info_from_codeword(const float* cw,
                               unsigned N,
                               const uint8_t* isfrozen,
                               int systematic,
                               uint8_t* x,
                               uint8_t* out)
{
    for (unsigned i = 0; i < N; ++i) x[i] = (uint8_t)(fb(cw[i]) >> 31);
    if (!systematic) polar_transform(x, N); /* fastssc_avx_float.cpp:944-947 */
    pack_info(x, N, isfrozen, out);
}

static int check_args(unsigned N, const uint32_t* frozen, unsigned nf)
{
    if (N < 8 || (N & (N - 1)) || nf > N) return -1;
    for (unsigned i = 0; i < nf; ++i) {
        if (frozen[i] >= N) return -1;
        if (i && frozen[i] <= frozen[i - 1]) return -1;
    }
    return 0;
}

/* Node-type census of the Fast-SSC tree, pre-order; returns node count or <0. */
int orc_sc_tree(uint32_t N, const uint32_t* frozen, uint32_t nf, int32_t* types, int32_t* sizes, int maxn);

static int sc_walk(const sc_node* x, int32_t* t, int32_t* s, int k, int maxn)
{
    if (!x) return k;
    if (k < maxn) { t[k] = x->type; s[k] = (int32_t)x->n; }
    k++;
    k = sc_walk(x->l, t, s, k, maxn);
    return sc_walk(x->r, t, s, k, maxn);
}

int orc_sc_tree(uint32_t N, const uint32_t* frozen, uint32_t nf, int32_t* types, int32_t* sizes, int maxn)
{
    if (check_args(N, frozen, nf)) return -1;
    int err = 0;
    sc_node* root = sc_create(frozen, nf, N, &err);
    if (!root) return err ? err : -1;
    int k = sc_walk(root, types, sizes, 0, maxn);
    sc_free(root);
    return k;
}

/* Batched Fast-SSC decode.  info: F x ceil(K/8); ok: F (nullable);
 * softcw: F x N floats (nullable) = Decoder::getSoftCodeword. */
int orc_sc_decode(uint32_t N,
                  const uint32_t* frozen,
                  uint32_t nf,
                  int systematic,
                  int crc,
                  const float* llr,
                  uint64_t F,
                  uint8_t* info,
                  uint8_t* ok,
                  float* softcw)
{
    if (check_args(N, frozen, nf)) return -1;
    int err = 0;
    sc_node* root = sc_create(frozen, nf, N, &err);
    if (!root) return err ? err : -1;
    const unsigned kb = (N - nf + 7) / 8;
    uint8_t* isf = (uint8_t*)calloc(N, 1);
    for (unsigned i = 0; i < nf; ++i) isf[frozen[i]] = 1;
    float* out = (float*)malloc(4 * N);
    float* scratch = (float*)malloc(4 * 2 * N);
    uint8_t* x = (uint8_t*)malloc(N);
    for (uint64_t f = 0; f < F; ++f) {
        sc_decode_node(root, llr + f * N, out, scratch);
        uint8_t* o = info + f * kb;
        info_from_codeword(out, N, isf, systematic, x, o);
        int r = orc_crc(crc, 0, o, (int)kb);
        if (ok) ok[f] = (uint8_t)(r > 0);
        if (softcw) memcpy(softcw + f * N, out, 4 * N);
    }
    free(out); free(scratch); free(x); free(isf);
    sc_free(root);
    return 0;
}

/* ================================================================== */
/* SCL (SclAvxFloat)            src/polarcode/decoding/scl_avx_float.cpp */
/* ================================================================== */
enum { SL_R0 = 0, SL_R1, SL_REP, SL_SPC, SL_RATER };

typedef struct sl_node {
    int type;
    unsigned n, s; /* size and stage (log2 n) */
    struct sl_node *l, *r;
} sl_node;

static void sl_free(sl_node* x)
{
    if (!x) return;
    sl_free(x->l);
    sl_free(x->r);
    free(x);
}

/* SclAvx::createDecoder, scl_avx_float.cpp:624-651 */
static sl_node* sl_create(const uint32_t* f, unsigned nf, unsigned n)
{
    sl_node* x = (sl_node*)calloc(1, sizeof(sl_node));
    x->n = n;
    x->s = (unsigned)__builtin_ctz(n);
    if (nf == 0) { x->type = SL_R1; return x; }
    if (nf == n) { x->type = SL_R0; return x; }
    if (nf == n - 1 && n < 8) { x->type = SL_REP; return x; }
    if (nf == 1) { x->type = SL_SPC; return x; }
    x->type = SL_RATER;
    unsigned h = n / 2, nl, nr;
    uint32_t* lf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    uint32_t* rf = (uint32_t*)malloc(sizeof(uint32_t) * (nf + 1));
    split_frozen(f, nf, h, lf, &nl, rf, &nr);
    x->l = sl_create(lf, nl, h);
    x->r = sl_create(rf, nr, h);
    free(lf);
    free(rf);
    return x;
}

typedef struct {
    unsigned L, S, P;          /* list size, stage count (log2N+1), active paths */
    float* llr[2];             /* [L][S][stride] current / next */
    float* bit[2];
    float* lbit[2];
    float metric[2][64];
    int cur;
    unsigned stride;           /* max(8, N) floats per stage slot */
    /* candidate scratch */
    float cm[8 * 64];
    unsigned cidx[8 * 64];
    unsigned flips[8 * 64][4];
    unsigned nflip[8 * 64];
    float cres[8 * 64];        /* repetition results */
    unsigned nfl_copy[8 * 64], fl_copy[8 * 64][4];
    unsigned* tidx;            /* >= N */
    float* tmp;                /* >= N + 8 */
} sl_state;

#define SLP(st, arr, which, p, s) ((st)->arr[which] + ((size_t)(p) * (st)->S + (s)) * (st)->stride)

/* simplePartialSortDescending(Indices, Values, n, size), include/polarcode/arrayfuncs.h:161-183:
 * swap-selection sort, lim = min(size-1, n) passes, first strictly-greater wins. */
static void partial_sort_desc(unsigned* idx, float* v, unsigned n, unsigned size)
{
    for (unsigned i = 0; i < size; ++i) idx[i] = i;
    unsigned lim = size - 1 < n ? size - 1 : n;
    for (unsigned i = 0; i < lim; ++i) {
        unsigned b = i;
        for (unsigned j = i + 1; j < size; ++j)
            if (v[j] > v[b]) b = j;
        float tv = v[i]; v[i] = v[b]; v[b] = tv;
        unsigned ti = idx[i]; idx[i] = idx[b]; idx[b] = ti;
    }
}

/* findWeakLlrs(Indices, Values, size, n), arrayfuncs.h:209-231: ascending, strict '<' */
static void find_weak(unsigned* idx, float* v, unsigned size, unsigned n)
{
    for (unsigned i = 0; i < size; ++i) idx[i] = i;
    unsigned lim = size - 1 < n ? size - 1 : n;
    for (unsigned i = 0; i < lim; ++i) {
        unsigned b = i;
        for (unsigned j = i + 1; j < size; ++j)
            if (v[j] < v[b]) b = j;
        float tv = v[i]; v[i] = v[b]; v[b] = tv;
        unsigned ti = idx[i]; idx[i] = idx[b]; idx[b] = ti;
    }
}

/* PathList::duplicatePath into the next list (eager copy of stages >= s; the
 * reference's lazy ref-counted copy, datapool.txx:86-120, is observably identical) */
static void sl_dup(sl_state* st, unsigned dst, unsigned src, unsigned s)
{
    int c = st->cur, x = 1 - c;
    for (unsigned k = s; k < st->S; ++k) {
        size_t bytes = 4 * (size_t)((1u << k) < 8 ? 8 : (1u << k));
        memcpy(SLP(st, llr, x, dst, k), SLP(st, llr, c, src, k), bytes);
        memcpy(SLP(st, bit, x, dst, k), SLP(st, bit, c, src, k), bytes);
        memcpy(SLP(st, lbit, x, dst, k), SLP(st, lbit, c, src, k), bytes);
    }
}

static void sl_select_and_switch(sl_state* st, const sl_node* x, unsigned k)
{
    /* k candidates per path; newPathCount = min(k*P, L); sort; duplicate; switch */
    const unsigned P = st->P, size = k * P;
    const unsigned np = size < st->L ? size : st->L;
    partial_sort_desc(st->cidx, st->cm, np, size);
    for (unsigned p = 0; p < np; ++p) sl_dup(st, p, st->cidx[p] / k, x->s);
    st->cur = 1 - st->cur;
    st->P = np;
    for (unsigned p = 0; p < np; ++p) st->metric[st->cur][p] = st->cm[p];
}

static void sl_leaf(sl_state* st, const sl_node* x)
{
    const unsigned n = x->n, s = x->s, P = st->P;
    const unsigned nn = n < 8 ? 8 : n;
    int c = st->cur;
    switch (x->type) {
    case SL_R0: /* :316-337, no re-sort */
        for (unsigned p = 0; p < P; ++p) {
            float* l = SLP(st, llr, c, p, s);
            float* b = SLP(st, bit, c, p, s);
            for (unsigned i = n; i < 8; ++i) l[i] = 0.0f;
            float pun[8] = { 0, 0, 0, 0, 0, 0, 0, 0 };
            for (unsigned i = 0; i < nn; i += 8)
                for (unsigned j = 0; j < 8; ++j) {
                    b[i + j] = INFINITY;
                    pun[j] = pun[j] + minps(l[i + j], 0.0f);
                }
            st->metric[c][p] += reduce_add8(pun);
        }
        return;
    case SL_R1: /* :353-413 */
        for (unsigned p = 0; p < P; ++p) {
            float m = st->metric[c][p];
            float* l = SLP(st, llr, c, p, s);
            for (unsigned i = n; i < 8; ++i) l[i] = INFINITY;
            for (unsigned i = 0; i < nn; ++i) st->tmp[i] = fabs_(l[i]);
            find_weak(st->tidx, st->tmp, n, 2);
            st->cm[4 * p] = m;
            st->cm[4 * p + 1] = m - st->tmp[0];
            st->cm[4 * p + 2] = m - st->tmp[1];
            st->cm[4 * p + 3] = m - st->tmp[0] - st->tmp[1];
            st->nflip[4 * p] = 0;
            st->nflip[4 * p + 1] = 1; st->flips[4 * p + 1][0] = st->tidx[0];
            st->nflip[4 * p + 2] = 1; st->flips[4 * p + 2][0] = st->tidx[1];
            st->nflip[4 * p + 3] = 2; st->flips[4 * p + 3][0] = st->tidx[0];
            st->flips[4 * p + 3][1] = st->tidx[1];
        }
        break;
    case SL_REP: /* :428-481 (n < 8 only) */
        for (unsigned p = 0; p < P; ++p) {
            float m = st->metric[c][p];
            float* l = SLP(st, llr, c, p, s);
            for (unsigned i = n; i < 8; ++i) l[i] = 0.0f;
            float z[8], o[8], r[8];
            for (unsigned j = 0; j < 8; ++j) {
                z[j] = 0.0f + minps(l[j], 0.0f);
                o[j] = 0.0f + maxps(l[j], 0.0f);
                r[j] = 0.0f + l[j];
            }
            float res = fabsf(reduce_add8(r));
            st->cres[2 * p] = res;
            st->cres[2 * p + 1] = -res;
            st->cm[2 * p] = m + reduce_add8(z);
            st->cm[2 * p + 1] = m - reduce_add8(o);
        }
        {
            unsigned size = 2 * P, np = size < st->L ? size : st->L;
            float res_copy[8 * 64];
            memcpy(res_copy, st->cres, sizeof(float) * size);
            sl_select_and_switch(st, x, 2);
            for (unsigned p = 0; p < np; ++p) {
                float* b = SLP(st, bit, st->cur, p, s);
                for (unsigned i = 0; i < nn; ++i) b[i] = res_copy[st->cidx[p]];
            }
        }
        return;
    case SL_SPC: /* :498-621 */
        for (unsigned p = 0; p < P; ++p) {
            float m = st->metric[c][p];
            float* l = SLP(st, llr, c, p, s);
            for (unsigned i = n; i < 8; ++i) l[i] = INFINITY;
            uint32_t par = 0;
            for (unsigned i = 0; i < nn; ++i) {
                par ^= fb(l[i]);
                st->tmp[i] = fabs_(l[i]);
            }
            find_weak(st->tidx, st->tmp, n, 4);
            const float* T = st->tmp;
            const unsigned* I = st->tidx;
            unsigned* nfl = st->nflip + 8 * p;
            unsigned(*fl)[4] = st->flips + 8 * p;
            float pinv;
            if (par & 0x80000000u) {
                pinv = 0.0f;
                m -= T[0];
                nfl[0] = 1; fl[0][0] = I[0];
                nfl[1] = 0; nfl[2] = 0; nfl[3] = 0;
                nfl[4] = 1; fl[4][0] = I[0];
                nfl[5] = 1; fl[5][0] = I[0];
                nfl[6] = 1; fl[6][0] = I[0];
                nfl[7] = 0;
            } else {
                pinv = 1.0f;
                nfl[0] = 0;
                nfl[1] = 1; fl[1][0] = I[0];
                nfl[2] = 1; fl[2][0] = I[0];
                nfl[3] = 1; fl[3][0] = I[0];
                nfl[4] = 0; nfl[5] = 0; nfl[6] = 0;
                nfl[7] = 1; fl[7][0] = I[0];
            }
            float* cm = st->cm + 8 * p;
            cm[0] = m;
            cm[1] = m - pinv * T[0] - T[1];
            cm[2] = m - pinv * T[0] - T[2];
            cm[3] = m - pinv * T[0] - T[3];
            cm[4] = m - T[1] - T[2];
            cm[5] = m - T[1] - T[3];
            cm[6] = m - T[2] - T[3];
            cm[7] = m - pinv * T[0] - T[1] - T[2] - T[3];
            fl[1][nfl[1]++] = I[1];
            fl[2][nfl[2]++] = I[2];
            fl[3][nfl[3]++] = I[3];
            fl[4][nfl[4]++] = I[1]; fl[4][nfl[4]++] = I[2];
            fl[5][nfl[5]++] = I[1]; fl[5][nfl[5]++] = I[3];
            fl[6][nfl[6]++] = I[2]; fl[6][nfl[6]++] = I[3];
            fl[7][nfl[7]++] = I[1]; fl[7][nfl[7]++] = I[2]; fl[7][nfl[7]++] = I[3];
        }
        break;
    default:
        return;
    }
    /* R1 / SPC: select survivors, bits = copy of the source LLR + flips */
    {
        const unsigned k = x->type == SL_R1 ? 4 : 8;
        const unsigned size = k * P, np = size < st->L ? size : st->L;
        unsigned* nfl_copy = st->nfl_copy;
        unsigned(*fl_copy)[4] = st->fl_copy;
        memcpy(nfl_copy, st->nflip, sizeof(unsigned) * size);
        memcpy(fl_copy, st->flips, sizeof(unsigned) * 4 * size);
        sl_select_and_switch(st, x, k);
        for (unsigned p = 0; p < np; ++p) {
            unsigned src = st->cidx[p];
            const float* l = SLP(st, llr, st->cur, p, s);
            float* b = SLP(st, bit, st->cur, p, s);
            memcpy(b, l, 4 * nn);
            for (unsigned q = 0; q < nfl_copy[src]; ++q) {
                unsigned i = fl_copy[src][q];
                b[i] = bf(fb(b[i]) ^ 0x80000000u);
            }
        }
    }
}

static void sl_decode_node(sl_state* st, const sl_node* x)
{
    if (x->type != SL_RATER) {
        sl_leaf(st, x);
        return;
    }
    /* RateRNode / ShortRateRNode::decode, scl_avx_float.cpp:229-307 */
    const unsigned h = x->n / 2, cs = x->s - 1, ps = x->s;
    for (unsigned p = 0; p < st->P; ++p) {
        const float* in = SLP(st, llr, st->cur, p, ps);
        float* o = SLP(st, llr, st->cur, p, cs);
        for (unsigned i = 0; i < h; ++i) o[i] = polar_f(in[i], in[h + i]);
    }
    sl_decode_node(st, x->l);
    for (unsigned p = 0; p < st->P; ++p) {
        /* prepareRightDecoding: Bit <-> LeftBit at the child stage */
        float* b = SLP(st, bit, st->cur, p, cs);
        float* lb = SLP(st, lbit, st->cur, p, cs);
        for (unsigned i = 0; i < (h < 8 ? 8 : h); ++i) { float t = b[i]; b[i] = lb[i]; lb[i] = t; }
        const float* in = SLP(st, llr, st->cur, p, ps);
        float* o = SLP(st, llr, st->cur, p, cs);
        for (unsigned i = 0; i < h; ++i) o[i] = polar_g(in[i], in[h + i], lb[i]);
    }
    sl_decode_node(st, x->r);
    for (unsigned p = 0; p < st->P; ++p) {
        const float* lb = SLP(st, lbit, st->cur, p, cs);
        const float* rb = SLP(st, bit, st->cur, p, cs);
        float* o = SLP(st, bit, st->cur, p, ps);
        for (unsigned i = 0; i < h; ++i) {
            o[i] = fxor(lb[i], rb[i]);
            o[h + i] = rb[i];
        }
    }
}

/* Batched SCL decode.  carry != 0 reproduces the reference's cross-frame carry of
 * path 0's metric (PathList::clear/setFirstPath never reset mMetric,
 * scl_avx_float.cpp:48-56,103-109); carry == 0 = a freshly
 * constructed decoder per frame (what the GPU path implements).
 * metrics: F x L (nullable), pathcount: F (nullable), pathbits: F x L x N/8 (nullable). */
int orc_scl_decode(uint32_t N,
                   uint32_t L,
                   const uint32_t* frozen,
                   uint32_t nf,
                   int systematic,
                   int crc,
                   int carry,
                   const float* llr,
                   uint64_t F,
                   uint8_t* info,
                   uint8_t* ok,
                   float* metrics,
                   uint32_t* pathcount,
                   uint8_t* pathbits)
{
    if (check_args(N, frozen, nf) || L < 1 || L > 64) return -1;
    sl_node* root = sl_create(frozen, nf, N);
    sl_state* st = (sl_state*)calloc(1, sizeof(sl_state));
    st->L = L;
    st->S = (unsigned)__builtin_ctz(N) + 1;
    st->stride = N < 8 ? 8 : N;
    st->tidx = (unsigned*)calloc(N + 8, sizeof(unsigned));
    st->tmp = (float*)calloc(N + 8, sizeof(float));
    size_t tot = (size_t)L * st->S * st->stride;
    for (int w = 0; w < 2; ++w) {
        st->llr[w] = (float*)calloc(tot, 4);
        st->bit[w] = (float*)calloc(tot, 4);
        st->lbit[w] = (float*)calloc(tot, 4);
    }
    const unsigned kb = (N - nf + 7) / 8, top = st->S - 1;
    uint8_t* isf = (uint8_t*)calloc(N, 1);
    for (unsigned i = 0; i < nf; ++i) isf[frozen[i]] = 1;
    uint8_t* x = (uint8_t*)malloc(N);
    uint8_t* o = (uint8_t*)malloc(kb + 8);
    float carried = 0.0f;
    for (uint64_t f = 0; f < F; ++f) {
        st->cur = 0;
        st->P = 1;
        st->metric[0][0] = carry ? carried : 0.0f;
        memcpy(SLP(st, llr, 0, 0, top), llr + f * N, 4 * N);
        sl_decode_node(st, root);
        const unsigned P = st->P;
        /* extractBestPath, scl_avx_float.cpp:711-750 */
        int found = 0;
        for (unsigned p = 0; p < P && !found; ++p) {
            info_from_codeword(SLP(st, bit, st->cur, p, top), N, isf, systematic, x, o);
            if (orc_crc(crc, 0, o, (int)kb) > 0) found = 1;
        }
        if (!found) info_from_codeword(SLP(st, bit, st->cur, 0, top), N, isf, systematic, x, o);
        memcpy(info + f * kb, o, kb);
        if (ok) ok[f] = (uint8_t)found;
        carried = st->metric[st->cur][0];
        if (pathcount) pathcount[f] = P;
        for (unsigned p = 0; p < L; ++p) {
            if (metrics) metrics[f * L + p] = p < P ? st->metric[st->cur][p] : 0.0f;
            if (pathbits) {
                uint8_t* pb = pathbits + (f * L + p) * (N / 8);
                memset(pb, 0, N / 8);
                if (p < P) {
                    const float* b = SLP(st, bit, st->cur, p, top);
                    for (unsigned i = 0; i < N; ++i)
                        if (fb(b[i]) >> 31) pb[i / 8] |= (uint8_t)(0x80u >> (i % 8));
                }
            }
        }
    }
    for (int w = 0; w < 2; ++w) { free(st->llr[w]); free(st->bit[w]); free(st->lbit[w]); }
    free(st->tidx); free(st->tmp);
    free(st); free(isf); free(x); free(o);
    sl_free(root);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Encoder: ButterflyFipPacked::encode (butterfly_fip_packed.cpp:45-58) */
/* ------------------------------------------------------------------ */
int orc_encode(uint32_t N,
               const uint32_t* frozen,
               uint32_t nf,
               int systematic,
               int crc,
               const uint8_t* info,
               uint64_t F,
               uint8_t* code)
{
    if (check_args(N, frozen, nf)) return -1;
    const unsigned K = N - nf, kb = (K + 7) / 8;
    uint8_t* isf = (uint8_t*)calloc(N, 1);
    for (unsigned i = 0; i < nf; ++i) isf[frozen[i]] = 1;
    uint8_t* u = (uint8_t*)malloc(N);
    uint8_t* d = (uint8_t*)malloc(kb + 8);
    for (uint64_t f = 0; f < F; ++f) {
        memcpy(d, info + f * kb, kb);
        if (crc > 0) orc_crc(crc, 1, d, (int)(K / 8));
        unsigned j = 0;
        for (unsigned i = 0; i < N; ++i) {
            u[i] = 0;
            if (!isf[i]) { u[i] = (d[j / 8] >> (7 - j % 8)) & 1; ++j; }
        }
        polar_transform(u, N);
        if (systematic) {
            for (unsigned i = 0; i < N; ++i) if (isf[i]) u[i] = 0;
            polar_transform(u, N);
        }
        uint8_t* c = code + f * (N / 8);
        memset(c, 0, N / 8);
        for (unsigned i = 0; i < N; ++i) if (u[i]) c[i / 8] |= (uint8_t)(0x80u >> (i % 8));
    }
    free(isf); free(u); free(d);
    return 0;
}

/* ------------------------------------------------------------------ */
/* Bhattacharyya construction  src/polarcode/construction/bhattacharrya.cpp:39-82 */
/* ------------------------------------------------------------------ */
int orc_frozen_bits_bb(uint32_t N, uint32_t K, float dsnr, uint32_t* out)
{
    if (N < 2 || (N & (N - 1)) || K > N) return -1;
    float lin = (float)pow(10.0, dsnr / 10.0);
    float init = (float)exp(-2.0 * lin * K / N);
    double* z = (double*)malloc(sizeof(double) * N);
    int* perm = (int*)malloc(sizeof(int) * N);
    z[0] = init;
    int n = __builtin_ctz(N);
    for (int stage = n - 1; stage >= 0; --stage) {
        unsigned B = 1u << stage;
        for (unsigned j = 0; j < N; j += 2 * B) {
            double T = z[j];
            z[j + B] = T * T;
            z[j] = 2 * T - z[j + B];
        }
    }
    /* trackingSorter::stableSortDescending (arrayfuncs.cpp:93-107): insertion sort */
    for (unsigned i = 0; i < N; ++i) perm[i] = (int)i;
    for (int i = 1; i < (int)N; ++i) {
        double xv = z[i];
        int y = perm[i], j = i - 1;
        while (j >= 0 && z[j] < xv) { z[j + 1] = z[j]; perm[j + 1] = perm[j]; j--; }
        z[j + 1] = xv;
        perm[j + 1] = y;
    }
    unsigned nf = N - K;
    for (unsigned i = 0; i < nf; ++i) out[i] = (uint32_t)perm[i];
    /* std::sort ascending */
    for (unsigned i = 1; i < nf; ++i) {
        uint32_t v = out[i];
        int j = (int)i - 1;
        while (j >= 0 && out[j] > v) { out[j + 1] = out[j]; j--; }
        out[j + 1] = v;
    }
    free(z); free(perm);
    return (int)nf;
}

/* single-thread throughput of this restatement (cw/s) */
double orc_bench(uint32_t N, uint32_t L, const uint32_t* frozen, uint32_t nf,
                 const float* llr, uint64_t F, int reps)
{
    const unsigned kb = (N - nf + 7) / 8;
    uint8_t* info = (uint8_t*)malloc((size_t)F * kb);
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (int r = 0; r < reps; ++r) {
        if (L <= 1) orc_sc_decode(N, frozen, nf, 1, -1, llr, F, info, NULL, NULL);
        else orc_scl_decode(N, L, frozen, nf, 1, -1, 0, llr, F, info, NULL, NULL, NULL, NULL);
    }
    clock_gettime(CLOCK_MONOTONIC, &b);
    free(info);
    double s = (b.tv_sec - a.tv_sec) + 1e-9 * (b.tv_nsec - a.tv_nsec);
    return (double)F * reps / s;
}

/* KAT hooks: the reference's 8-lane F / G / CombineBitsShort on plain arrays
 * (test/polarcode/decodingtest.cpp:462-494 exercises these). */
void orc_f(const float* in, float* out, uint32_t h)
{
    for (uint32_t i = 0; i < h; ++i) out[i] = polar_f(in[i], in[h + i]);
}
void orc_g(const float* in, const float* bits, float* out, uint32_t h)
{
    for (uint32_t i = 0; i < h; ++i) out[i] = polar_g(in[i], in[h + i], bits[i]);
}
void orc_combine_short(const float* l, const float* r, float* out, uint32_t h)
{
    for (uint32_t i = 0; i < 8; ++i) out[i] = 0.0f;
    for (uint32_t i = 0; i < h; ++i) {
        out[i] = fxor(l[i], r[i]);
        out[h + i] = r[i];
    }
}

/* ------------------------------------------------------------------ */
/* Puncturer  src/polarcode/puncturer.cpp:23-89, include/polarcode/puncturer.h:60-99 */
/* ------------------------------------------------------------------ */
/* Kept parent positions for Puncturer(E, frozen): parent = next power of two >= E,
 * the first parent-E entries of `frozen` (as given) removed from [0, parent).
 * Returns the number of kept positions, -1 if the frozen set is too small. */
int orc_puncturer(uint32_t E, const uint32_t* frozen, uint32_t nf, uint32_t* parent, uint32_t* pos)
{
    uint32_t N = 1;
    while (N < E) N <<= 1;                 /* round_up_power_of_two, E >= 1 */
    uint32_t np = N - E, k = 0;
    if (np > nf) return -1;                /* std::out_of_range, puncturer.cpp:57-60 */
    /* std::set_difference over ascending ranges (written as a membership test) */
    for (uint32_t x = 0; x < N; ++x) {
        int gone = 0;
        for (uint32_t j = 0; j < np; ++j) if (frozen[j] == x) { gone = 1; break; }
        if (!gone) pos[k++] = x;
    }
    *parent = N;
    return (int)k;
}

/* depuncture (puncturer.h:92-99): zero-fill, then scatter; F frames */
void orc_depuncture(uint32_t E, uint32_t N, const uint32_t* pos, const float* in, uint64_t F, float* out)
{
    for (uint64_t f = 0; f < F; ++f) {
        for (uint32_t i = 0; i < N; ++i) out[f * N + i] = 0.0f;
        for (uint32_t k = 0; k < E; ++k) out[f * N + pos[k]] = in[f * E + k];
    }
}

/* puncturePacked (puncturer.cpp:71-89): MSB-first bits, one frame */
void orc_puncture_packed(uint32_t E, const uint32_t* pos, const uint8_t* in, uint8_t* out)
{
    for (uint32_t b = 0; b < E / 8; ++b) {
        uint8_t o = 0;
        for (uint32_t i = 0; i < 8; ++i) {
            uint32_t p = pos[8 * b + i];
            if ((in[p / 8] >> (7 - p % 8)) & 1) o |= (uint8_t)(0x80u >> i);
        }
        out[b] = o;
    }
}
