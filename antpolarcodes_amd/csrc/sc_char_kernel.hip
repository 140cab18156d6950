// sc_char_kernel.hip -- batched 8-bit fixed-point Fast-SSC polar decoding
// (the reference's FastSscFipChar, src/polarcode/decoding/fastssc_fip_char.cpp) on
// CDNA4 (gfx950).
//
// One codeword per wavefront walking the plan's flattened FastSscFip schedule
// (plan.cpp sc_char_emit) exactly like sc_kernel.hip.  LLRs are the reference's
// signed bytes; each stage element is kept sign-extended in a 32-bit LDS word so
// every byte operation of fip_char.h (saturating add/sub, abs, min/max, sign) is
// one or two 32-bit VALU ops with a clamp.  The channel frame is read straight from
// HBM at 1 byte per LLR (pcg_decode_i8) or as floats quantised on the fly with
// CharContainer::insertLlr's rounding (pcg_decode_f32 on a char plan).
//
// Only sign bits of the reference's "bit" bytes are observable downstream (G's
// blendv, Combine's XOR, the packing all read the sign), except inside the SPC /
// ZeroSPC leaves where a flip negates a byte: -0 and -(-128) keep their sign.  The
// codeword is therefore kept as packed sign bits, and the flip rule is applied to
// the byte it negates.  The 32-lane vector semantics of short nodes (n <= 32:
// padding, reduction trees, minpos over the padded vector) are reproduced per lane.
#include "kernels.hpp"
#include "plan.hpp"
#include "sc_common.hpp"
#include "wave.hpp"

namespace pcg {

namespace {

PCG_DEV int sat8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }

// FastSscFip::F_function_calc (fip_char.h:35-56)
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
// G_function_calc (fip_char.h:58-64): blendv(R + L, R - L, bit)
PCG_DEV int fip_g(int l, int r, uint32_t bit) { return sat8(bit ? r - l : r + l); }

// a flip "BitPtr[i] = -BitPtr[i]" changes the sign bit unless the byte is 0 or -128
PCG_DEV uint32_t flips_sign(int v) { return (v != 0 && v != -128) ? 1u : 0u; }

// channel readers: the frame in HBM, as int8 or as float quantised per
// CharContainer::insertLlr (bitcontainer.cpp:449-516)
struct ChanI8 {
    static constexpr bool kI8 = true;
    const int8_t* y;
    PCG_DEV int operator[](uint32_t i) const { return y[i]; }
};
struct ChanF32 {
    static constexpr bool kI8 = false;
    const float* y;
    uint32_t large; // N >= 32: convert_f32_to_int8_large, else vectorizedFtoC
    PCG_DEV int operator[](uint32_t i) const
    {
        const float x = y[i];
        if (large) { // _mm256_cvtps_epi32 (NaN / |x| >= 2^31 -> INT32_MIN) + saturating packs
            if (!(x < 2147483648.0f) || x < -2147483648.0f)
                return -128;
            const float r = __builtin_rintf(x);
            return r <= -128.0f ? -128 : (r >= 127.0f ? 127 : (int)r);
        }
        float v = x > -128.0f ? x : -128.0f; // _mm256_max_ps(x, -128): NaN -> -128
        v = v < 127.0f ? v : 127.0f;
        return (int)__builtin_rintf(v);
    }
};
struct StageI {
    const int* x;
    PCG_DEV int operator[](uint32_t i) const { return x[i]; }
};

// saturating reduction tree of reduce_adds_epi8 (avxconvenience.h:92-101) over lanes
// 0..31: pairs (i, i+16), (i, i+8), ..., (i, i+1); valid in lane 0
PCG_DEV int reduce_adds32(int v)
{
    for (int k = 16; k >= 1; k >>= 1)
        v = sat8(v + __shfl_down(v, k, 64));
    return __shfl(v, 0, 64);
}

// first index of the smallest value over the wave (ties -> lowest index)
PCG_DEV void argmin_i(int& v, uint32_t& i)
{
    for (int d = 32; d >= 1; d >>= 1) {
        const int ov = __shfl_xor(v, d, 64);
        const uint32_t oi = __shfl_xor(i, d, 64);
        if (ov < v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

// SpcDecoder / ZeroSpcDecoder (n > 32) minimum search: per 32-byte vector minpos of |x|,
// kept only if strictly below the running minimum that starts at 127
// (fastssc_fip_char.cpp:287-297, 336-350) = first index of the global minimum if that
// minimum is < 127, else index 0.
template <typename Val>
PCG_DEV void spc_long(Val val, uint32_t n, uint32_t lane, uint32_t& mi, uint32_t& par)
{
    int mv = 1 << 20;
    mi = 0xffffffffu;
    par = 0;
    for (uint32_t i = lane; i < n; i += 64) {
        const int v = val(i);
        par ^= v < 0 ? 1u : 0u;
        const int a = v < 0 ? -v : v; // |x| as an unsigned byte (|-128| = 128)
        if (a < mv) {
            mv = a;
            mi = i;
        }
    }
    argmin_i(mv, mi);
    par = wave_xor(par) & 1u;
    if (mv >= 127)
        mi = 0;
}

// minpos_epu8 over one padded 32-byte vector (lanes 0..31 hold the bytes): first lane
// of the smallest |x| (ShortSpcDecoder / ShortZeroSpcDecoder)
PCG_DEV uint32_t minpos32(int v, uint32_t lane)
{
    int a = lane < 32 ? (v < 0 ? -v : v) : (1 << 20);
    uint32_t i = lane;
    argmin_i(a, i);
    return i;
}

template <typename Src>
PCG_DEV void leaf(uint32_t code, Src x, uint32_t n, uint32_t o, uint32_t* bits, uint32_t lane)
{
    switch (code) {
    case OP_C_R0: // 127 = bit 0
        fill_bits(bits, o, n, 0u, lane);
        break;
    case OP_C_R1:
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            put_bits(bits, o + b, n < 64 ? n : 64, i < n && x[i] < 0);
        }
        break;
    case OP_C_REP:  // lane-wise saturating accumulation over the vectors, then the tree
    case OP_C_DREP: {
        int acc = 0;
        if (lane < 32)
            for (uint32_t i = lane; i < n; i += 32)
                acc = sat8(acc + x[i]);
        if (code == OP_C_REP) {
            fill_bits(bits, o, n, reduce_adds32(acc) < 0 ? 1u : 0u, lane);
        } else { // half_reduce_adds_epi8 (avxconvenience.h:202-212): XOR butterflies 16..2
            for (int k = 16; k >= 2; k >>= 1)
                acc = sat8(acc + __shfl_xor(acc, k, 64));
            const uint32_t e = __shfl(acc, 0, 64) < 0 ? 1u : 0u, od = __shfl(acc, 1, 64) < 0 ? 1u : 0u;
            fill_pattern(bits, o, n, e | (od << 1), 2, lane);
        }
        break;
    }
    case OP_C_REPS: { // RepetitionPrepare pads with 0
        const int v = (lane < n) ? x[lane] : 0;
        fill_bits(bits, o, n, reduce_adds32(lane < 32 ? v : 0) < 0 ? 1u : 0u, lane);
        break;
    }
    case OP_C_SPC: {
        uint32_t mi, par;
        spc_long([&](uint32_t i) { return (int)x[i]; }, n, lane, mi, par);
        const uint32_t fl = par ? flips_sign(x[mi]) : 0u;
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            uint32_t s = (i < n && x[i] < 0) ? 1u : 0u;
            if (i == mi)
                s ^= fl;
            put_bits(bits, o + b, n < 64 ? n : 64, s != 0);
        }
        break;
    }
    case OP_C_SPCS: { // SpcPrepare pads with 127
        const int v = lane < n ? x[lane] : 127;
        const uint32_t par = wave_xor((lane < 32 && v < 0) ? 1u : 0u) & 1u;
        const uint32_t mi = minpos32(v, lane);
        const int vm = __shfl(v, (int)mi, 64);
        const uint32_t fl = par ? flips_sign(vm) : 0u;
        put_bits(bits, o, n, lane < n && (((v < 0) ? 1u : 0u) ^ (lane == mi ? fl : 0u)) != 0);
        break;
    }
    case OP_C_ZSPC: { // G0 of the halves, SPC on it, output to both halves
        const uint32_t h = n / 2;
        uint32_t mi, par;
        spc_long([&](uint32_t i) { return sat8(x[i] + x[i + h]); }, h, lane, mi, par);
        const uint32_t fl = par ? flips_sign(sat8(x[mi] + x[mi + h])) : 0u;
        for (uint32_t b = 0; b < h; b += 64) {
            const uint32_t i = b + lane;
            uint32_t s = (i < h && sat8(x[i] + x[i + h]) < 0) ? 1u : 0u;
            if (i == mi)
                s ^= fl;
            const uint32_t c = h < 64 ? h : 64;
            put_bits(bits, o + b, c, s != 0);
            put_bits(bits, o + h + b, c, s != 0);
        }
        break;
    }
    case OP_C_ZSPCS: { // lanes >= h padded with 127 (fastssc_fip_char.cpp:372)
        const uint32_t h = n / 2;
        const int v = lane < h ? sat8(x[lane] + x[lane + h]) : 127;
        const uint32_t par = wave_xor((lane < 32 && v < 0) ? 1u : 0u) & 1u;
        const uint32_t mi = minpos32(v, lane);
        const int vm = __shfl(v, (int)mi, 64);
        const uint32_t fl = par ? flips_sign(vm) : 0u;
        const bool s = lane < h && (((v < 0) ? 1u : 0u) ^ (lane == mi ? fl : 0u)) != 0;
        put_bits(bits, o, h, s);
        put_bits(bits, o + h, h, s);
        break;
    }
    case OP_C_ZONES: {
        const uint32_t h = n / 2;
        const bool s = lane < h && sat8(x[lane] + x[lane + h]) < 0;
        put_bits(bits, o, h, s);
        put_bits(bits, o + h, h, s);
        break;
    }
    default:
        break;
    }
}

// internal-node ops reading stage s from `x` (LDS or the channel frame in HBM)
template <typename Src>
PCG_DEV void inner(uint32_t code, Src x, uint32_t s, uint32_t o, int* alpha, uint32_t* bits, uint32_t lane)
{
    const uint32_t h = 1u << (s - 1);
    int* out = alpha + h;
    switch (code) {
    case OP_F:
        for (uint32_t i = lane; i < h; i += 64)
            out[i] = fip_f(x[i], x[i + h]);
        break;
    case OP_G:
        for (uint32_t i = lane; i < h; i += 64)
            out[i] = fip_g(x[i], x[i + h], get_bit(bits, o + i));
        break;
    case OP_G0:
        for (uint32_t i = lane; i < h; i += 64)
            out[i] = sat8(x[i] + x[i + h]);
        break;
    case OP_RONE: // simplifiedRightRateOneDecode(Short) :436-474
        for (uint32_t b = 0; b < h; b += 64) {
            const uint32_t i = b + lane;
            uint32_t lb = 0, rs = 0;
            if (i < h) {
                lb = get_bit(bits, o + i);
                rs = fip_g(x[i], x[i + h], lb) < 0 ? 1u : 0u;
            }
            const uint32_t c = h < 64 ? h : 64;
            put_bits(bits, o + b, c, (lb ^ rs) != 0);
            put_bits(bits, o + h + b, c, rs != 0);
        }
        break;
    default:
        break;
    }
}

template <int WAVES, typename Chan>
__global__ void __launch_bounds__(64 * WAVES) sc_char_kernel(KernelArgs a)
{
    extern __shared__ int smem_i[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t frame = (uint64_t)blockIdx.x * WAVES + wv;
    if (frame >= a.F)
        return;
    int* alpha = smem_i + wv * a.wave_lds_floats; // stage s at alpha + (1 << s)
    uint32_t* bits = reinterpret_cast<uint32_t*>(alpha + a.N);
    Chan y;
    if constexpr (Chan::kI8) {
        y.y = a.llr8 + frame * a.N;
    } else {
        y.y = a.llr + frame * a.N;
        y.large = a.N >= 32 ? 1u : 0u;
    }
    const uint32_t top = a.log2N;
    for (uint32_t k = 0; k < a.nops; ++k) {
        const uint32_t w = ld_const(a.ops, k);
        const uint32_t code = op_code(w), s = op_stage(w), o = op_off(w);
        if (code >= OP_C_R0) {
            if (s == top)
                leaf(code, y, 1u << s, o, bits, lane);
            else
                leaf(code, StageI{ alpha + (1u << s) }, 1u << s, o, bits, lane);
        } else if (code == OP_COMB || code == OP_COPY0) {
            sc_bits_op(code, s, o, bits, lane);
        } else {
            if (s == top)
                inner(code, y, s, o, alpha, bits, lane);
            else
                inner(code, StageI{ alpha + (1u << s) }, s, o, alpha, bits, lane);
        }
        wsync();
    }
    if (!a.systematic)
        polar_transform_bits(bits, a.N, lane);
    const uint32_t syn = emit_info(bits, a, frame, lane, true);
    if (lane == 0 && a.ok)
        a.ok[frame] = syn == 0 ? 1 : 0;
}

} // namespace

int launch_sc_char(const KernelArgs& a, hipStream_t stream)
{
    constexpr int WAVES = 4;
    const uint64_t blocks = (a.F + WAVES - 1) / WAVES;
    if (blocks == 0)
        return 0;
    const size_t lds = (size_t)WAVES * a.wave_lds_floats * sizeof(int);
    if (a.llr8)
        hipLaunchKernelGGL((sc_char_kernel<WAVES, ChanI8>), dim3((uint32_t)blocks), dim3(64 * WAVES), lds, stream, a);
    else
        hipLaunchKernelGGL((sc_char_kernel<WAVES, ChanF32>), dim3((uint32_t)blocks), dim3(64 * WAVES), lds, stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

} // namespace pcg
