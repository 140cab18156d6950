// sc_kernel.hip -- batched Fast-SSC ("SC") polar decoding on CDNA4 (gfx950).
//
// One codeword per wavefront.  The wave walks the plan's flattened op schedule
// (plan.hpp) -- the reference's recursive FastSscAvx node tree
// (src/polarcode/decoding/fastssc_avx_float.cpp) in decode order -- with every
// branch wave-uniform.  Per wave, LDS holds the LLR stage buffers alpha[s]
// (2^s floats at float offset 2^s, s < log2 N; the root stage is the channel
// LLR frame, read straight from HBM) and the codeword estimate as packed sign
// bits (N bits).  Only sign bits of the reference's float "bits" are observable
// (F/G use signs, Combine XORs whole words, the output packs sign bits), so the
// packed form is exact.  Every arithmetic step reproduces the AVX2 reference's
// lane order and sign-of-zero behaviour (see oracle/polar_oracle.c).
#include "plan.hpp"
#include "kernels.hpp"
#include "wave.hpp"
#include "sc_common.hpp"

namespace pcg {

namespace {

constexpr float FLT_MAX_ = 3.40282347e+38f;

// 8 lane partial sums of the reference (each lane from +0.0, chunks ascending,
// n < 8 padded with +0.0): valid in lanes 0..7.
template <typename Src>
PCG_DEV float lane_sum8(Src x, uint32_t n, uint32_t lane)
{
    float acc = 0.0f;
    if (lane < 8) {
        if (n < 8) {
            acc = acc + (lane < n ? x[lane] : 0.0f);
        } else {
            for (uint32_t i = lane; i < n; i += 8)
                acc = acc + x[i];
        }
    }
    return acc;
}

// reduce_add_ps: ((((((s0+s1)+s2)+s3)+s4)+s5)+s6)+s7   avxconvenience.h:256-272
PCG_DEV float reduce_add8(float s)
{
    float r = shfl(s, 0);
    for (int j = 1; j < 8; ++j)
        r = r + shfl(s, j);
    return r;
}

// _mm256_spc_right4_ps (avx_float.h:289-302) on v held in lanes 0..3 (also valid
// in any lane k: result for index k&3).  Returns the output float for k&3 (every lane
// whose |v| equals the minimum flips its sign when the XOR of the 4 signs is 1).
PCG_DEV float spc4_val(float v, uint32_t lane)
{
    const uint32_t k = lane & 3;
    const float v0 = shfl(v, 0), v1 = shfl(v, 1), v2 = shfl(v, 2), v3 = shfl(v, 3);
    const float m = minps(minps(fabs_(v0), fabs_(v2)), minps(fabs_(v1), fabs_(v3)));
    const uint32_t par = (fbits(v0) ^ fbits(v1) ^ fbits(v2) ^ fbits(v3)) & 0x80000000u;
    const float vk = k == 0 ? v0 : k == 1 ? v1 : k == 2 ? v2 : v3;
    return fxor(vk, fabs_(vk) == m ? par : 0u);
}
// ... and its output sign bit
PCG_DEV uint32_t spc4_sign(float v, uint32_t lane) { return sgn(spc4_val(v, lane)) >> 31; }

// Soft codeword (Decoder::getSoftCodeword, the root FloatContainer word for word): the
// leaf decoders' float outputs.  `val(i)` gives output i of the leaf's n outputs.
template <typename Fn>
PCG_DEV void soft_put(float* sw, uint32_t o, uint32_t n, uint32_t lane, Fn val)
{
    for (uint32_t i = lane; i < n; i += 64)
        sw[o + i] = val(i);
}

// Leaf decoders.  SOFT: also write the reference's float outputs to sw[o .. o+n)
// (oracle/polar_oracle.c sc_leaf, fastssc_avx_float.cpp:247-792).
template <bool SOFT, typename Src>
PCG_DEV void sc_leaf(uint32_t code, Src x, uint32_t n, uint32_t o, uint32_t* bits, uint32_t lane, float* sw)
{
    switch (code) {
    case OP_L_R0: // RateZeroDecoder: +INF bits
        fill_bits(bits, o, n, 0u, lane);
        if constexpr (SOFT)
            soft_put(sw, o, n, lane, [&](uint32_t) { return __builtin_inff(); });
        break;
    case OP_L_R1: // RateOneDecoder: bits = LLR
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            put_bits(bits, o + b, n < 64 ? n : 64, i < n && (sgn(x[i]) != 0));
        }
        if constexpr (SOFT)
            soft_put(sw, o, n, lane, [&](uint32_t i) { return x[i]; });
        break;
    case OP_L_REP: { // RepetitionDecoder :273-287
        const float S = reduce_add8(lane_sum8(x, n, lane));
        fill_bits(bits, o, n, sgn(S) >> 31, lane);
        if constexpr (SOFT)
            soft_put(sw, o, n, lane, [&](uint32_t) { return S; });
        break;
    }
    case OP_L_DREP: { // DoubleRepetitionDecoder :303-332
        const float s = lane_sum8(x, n, lane);
        float ev, od;
        const float s0 = shfl(s, 0), s1 = shfl(s, 1), s2 = shfl(s, 2), s3 = shfl(s, 3);
        const float s4 = shfl(s, 4), s5 = shfl(s, 5), s6 = shfl(s, 6), s7 = shfl(s, 7);
        if (n >= 8) {
            ev = (s0 + s4) + (s2 + s6);
            od = (s1 + s5) + (s3 + s7);
        } else {
            ev = ((s0 + s2) + s4) + s6;
            od = ((s1 + s3) + s5) + s7;
        }
        fill_pattern(bits, o, n, (sgn(ev) >> 31) | ((sgn(od) >> 31) << 1), 2, lane);
        if constexpr (SOFT)
            soft_put(sw, o, n, lane, [&](uint32_t i) { return (i & 1) ? od : ev; });
        break;
    }
    case OP_L_SPC: { // SpcDecoder :342-373 (n < 8 padded with +INF)
        float mv = __builtin_inff();
        uint32_t mi = 0xffffffffu, par = 0;
        for (uint32_t i = lane; i < n; i += 64) {
            const float v = x[i];
            par ^= fbits(v);
            const float a = fabs_(v);
            if (a < mv) {
                mv = a;
                mi = i;
            }
        }
        wave_argmin(mv, mi);
        par = wave_xor(par) & 0x80000000u;
        if (mi == 0xffffffffu)
            mi = 0;
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            uint32_t s = i < n ? sgn(x[i]) : 0u;
            if (i == mi)
                s ^= par;
            put_bits(bits, o + b, n < 64 ? n : 64, s != 0);
        }
        if constexpr (SOFT)
            soft_put(sw, o, n, lane, [&](uint32_t i) { return fxor(x[i], i == mi ? par : 0u); });
        break;
    }
    case OP_L_DSPC: { // DoubleSpcDecoder :425-466 (n >= 16)
        float mv = FLT_MAX_;
        uint32_t mi = 0, par = 0;
        if (lane < 8) {
            for (uint32_t i = lane; i < n; i += 8) {
                const float v = x[i];
                par ^= fbits(v);
                const float a = fabs_(v);
                if (!(a > mv)) { // _mm256_cmplt_ps is a GT compare: ties -> later index
                    mv = a;
                    mi = i;
                }
            }
        }
        float m[8];
        uint32_t id[8];
        uint32_t pe = 0, po = 0;
        for (int j = 0; j < 8; ++j) {
            m[j] = shfl(mv, j);
            id[j] = shfl(mi, j);
            const uint32_t p = shfl(par, j);
            if (j & 1)
                po ^= p;
            else
                pe ^= p;
        }
        const float ce = minps(minps(m[0], m[4]), minps(m[2], m[6]));
        const float co = minps(minps(m[1], m[5]), minps(m[3], m[7]));
        uint32_t ei = 0, oi = 0;
        for (int j = 6; j >= 0; j -= 2)
            if (m[j] == ce)
                ei = id[j];
        for (int j = 7; j >= 1; j -= 2)
            if (m[j] == co)
                oi = id[j];
        pe &= 0x80000000u;
        po &= 0x80000000u;
        for (uint32_t b = 0; b < n; b += 64) {
            const uint32_t i = b + lane;
            uint32_t s = i < n ? sgn(x[i]) : 0u;
            if (i == ei)
                s ^= pe;
            if (i == oi)
                s ^= po;
            put_bits(bits, o + b, n < 64 ? n : 64, s != 0);
        }
        if constexpr (SOFT)
            soft_put(sw, o, n, lane,
                     [&](uint32_t i) { return fxor(x[i], (i == ei ? pe : 0u) ^ (i == oi ? po : 0u)); });
        break;
    }
    case OP_L_DSPC8: { // DoubleSpcDecoderShort8 :473-488 (multi-flip on ties)
        const float v = lane < 8 ? x[lane] : 0.0f;
        float a[8];
        uint32_t pe = 0, po = 0;
        for (int j = 0; j < 8; ++j) {
            const float vj = shfl(v, j);
            a[j] = fabs_(vj);
            if (j & 1)
                po ^= fbits(vj);
            else
                pe ^= fbits(vj);
        }
        const float ce = minps(minps(a[0], a[4]), minps(a[2], a[6]));
        const float co = minps(minps(a[1], a[5]), minps(a[3], a[7]));
        const bool odd = lane & 1;
        const float ov = fxor(v, (fabs_(v) == (odd ? co : ce)) ? ((odd ? po : pe) & 0x80000000u) : 0u);
        put_bits(bits, o, 8, lane < 8 && sgn(ov) != 0);
        if constexpr (SOFT)
            if (lane < 8)
                sw[o + lane] = ov;
        break;
    }
    case OP_L_ZSPC8: { // ZeroSpcDecoderShort8 :556-565
        const uint32_t k = lane & 3;
        const float v = x[k] + x[k + 4];
        const float ov = spc4_val(v, lane);
        put_bits(bits, o, 8, lane < 8 && sgn(ov) != 0);
        if constexpr (SOFT)
            if (lane < 8)
                sw[o + lane] = ov; // both halves: the 4-lane result of lane & 3
        break;
    }
    case OP_L_TREP: { // TripleRepetitionDecoder :572-589
        const float sl = lane_sum8(x, n, lane);
        const float v = shfl(sl, lane & 3) + shfl(sl, (lane & 3) + 4);
        const float ov = spc4_val(v, lane);
        const uint32_t ob = sgn(ov) >> 31;
        if constexpr (SOFT) {
            const float o0 = shfl(ov, 0), o1 = shfl(ov, 1), o2 = shfl(ov, 2), o3 = shfl(ov, 3);
            soft_put(sw, o, n, lane, [&](uint32_t i) {
                const uint32_t k = i & 3;
                return k == 0 ? o0 : k == 1 ? o1 : k == 2 ? o2 : o3;
            });
        }
        uint32_t pat = 0;
        for (uint32_t k = 0; k < 4; ++k)
            pat |= (uint32_t)__builtin_amdgcn_readlane((int)ob, (int)k) << k;
        fill_pattern(bits, o, n, pat, 4, lane);
        break;
    }
    case OP_L_TYPE5:   // TypeFiveDecoder :762-792
    case OP_L_REPR1: { // RepetitionRateOneDecoderShort8 :718-739
        const float l = (code == OP_L_TYPE5) ? lane_sum8(x, n, lane) : (lane < 8 ? x[lane] : 0.0f);
        const uint32_t k = lane & 3;
        const float lk = shfl(l, k), lk4 = shfl(l, k + 4);
        const float r = polar_f(lk, lk4);
        const float R = (shfl(r, 0) + shfl(r, 1)) + (shfl(r, 2) + shfl(r, 3));
        const float g = polar_g(lk, lk4, sgn(R));
        const float og = (code == OP_L_TYPE5) ? spc4_val(g, lane) : g;
        const uint32_t ob = sgn(og) >> 31;
        if constexpr (SOFT) {
            // res[k] = +-1.0 with sign(R) ^ sign(o[k]), res[k+4] = o[k]; repeated over n
            float res[8];
            for (uint32_t q = 0; q < 4; ++q) {
                const float oq = shfl(og, (int)q);
                res[q] = ubits(((fbits(R) ^ fbits(oq)) & 0x80000000u) ^ fbits(1.0f));
                res[q + 4] = oq;
            }
            soft_put(sw, o, n, lane, [&](uint32_t i) {
                float r = res[0];
                for (uint32_t q = 1; q < 8; ++q)
                    r = (i & 7) == q ? res[q] : r;
                return r;
            });
        }
        uint32_t pat = 0;
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t oq = (uint32_t)__builtin_amdgcn_readlane((int)ob, (int)q);
            pat |= (oq ^ (sgn(R) >> 31)) << q;
            pat |= oq << (q + 4);
        }
        fill_pattern(bits, o, n, pat, 8, lane);
        break;
    }
    case OP_L_ZSPC: { // ZeroSpcDecoder :503-546 -- right half to both halves (Q1)
        const uint32_t h = n / 2;
        float mv = __builtin_inff();
        uint32_t mi = 0xffffffffu, par = 0;
        for (uint32_t i = lane; i < h; i += 64) {
            const float l = x[i] + x[h + i];
            par ^= fbits(l);
            const float a = fabs_(l);
            if (a < mv) {
                mv = a;
                mi = i;
            }
        }
        wave_argmin(mv, mi);
        par = wave_xor(par) & 0x80000000u;
        if (mi == 0xffffffffu)
            mi = 0;
        for (uint32_t b = 0; b < h; b += 64) {
            const uint32_t i = b + lane;
            uint32_t s = i < h ? sgn(x[h + i]) : 0u;
            if (i == mi)
                s ^= par;
            const uint32_t c = h < 64 ? h : 64;
            put_bits(bits, o + b, c, s != 0);
            put_bits(bits, o + h + b, c, s != 0);
        }
        if constexpr (SOFT)
            soft_put(sw, o, n, lane, [&](uint32_t i) {
                const uint32_t j = i < h ? i : i - h;
                return fxor(x[h + j], j == mi ? par : 0u);
            });
        break;
    }
    default:
        break;
    }
}

// COMB / COPY0 on the soft words: out[i] ^= out[i+h] as a full 32-bit XOR
// (avx_float.h:188-197), ZeroRNode's left := right (avx_float.h:199-204)
PCG_DEV void soft_bits_op(uint32_t code, uint32_t s, uint32_t o, float* sw, uint32_t lane)
{
    const uint32_t h = 1u << (s - 1);
    for (uint32_t i = lane; i < h; i += 64)
        sw[o + i] = (code == OP_COMB) ? ubits(fbits(sw[o + i]) ^ fbits(sw[o + h + i])) : sw[o + h + i];
}

// internal-node ops reading alpha[s] from `x` (LDS stage buffer or the frame in HBM)
template <bool SOFT, typename Src>
PCG_DEV void sc_inner(uint32_t code, Src x, uint32_t s, uint32_t o, float* alpha, uint32_t* bits, uint32_t lane,
                      float* sw)
{
    const uint32_t h = 1u << (s - 1);
    float* out = alpha + h;
    switch (code) {
    case OP_F:
        for (uint32_t i = lane; i < h; i += 64)
            out[i] = polar_f(x[i], x[i + h]);
        break;
    case OP_G:
        for (uint32_t i = lane; i < h; i += 64)
            out[i] = polar_g(x[i], x[i + h], get_bit(bits, o + i) << 31);
        break;
    case OP_G0:
        for (uint32_t i = lane; i < h; i += 64)
            out[i] = x[i] + x[i + h];
        break;
    case OP_RONE: // ROneNode::rightDecode :205-219
        for (uint32_t b = 0; b < h; b += 64) {
            const uint32_t i = b + lane;
            uint32_t lb = 0, rs = 0;
            if (i < h) {
                lb = get_bit(bits, o + i);
                const float r = polar_g(x[i], x[i + h], lb << 31);
                rs = sgn(r) >> 31;
            }
            const uint32_t c = h < 64 ? h : 64;
            put_bits(bits, o + b, c, (lb ^ rs) != 0);
            put_bits(bits, o + h + b, c, rs != 0);
        }
        if constexpr (SOFT) // outL = bitsL XOR r (word XOR), outR = r   (:205-219)
            for (uint32_t i = lane; i < h; i += 64) {
                const float bl = sw[o + i];
                const float r = polar_g(x[i], x[i + h], sgn(bl));
                sw[o + i] = ubits(fbits(bl) ^ fbits(r));
                sw[o + h + i] = r;
            }
        break;
    default:
        break;
    }
}

} // namespace

// SOFT: the wave also keeps the reference's float codeword (N floats of LDS after the
// packed bits) and writes it to a.soft (Decoder::getSoftCodeword).
template <int WAVES, bool SOFT>
__global__ void __launch_bounds__(64 * WAVES) sc_kernel(KernelArgs a)
{
    extern __shared__ float smem[];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t frame = (uint64_t)blockIdx.x * WAVES + wv;
    if (frame >= a.F)
        return;
    const uint32_t per_wave = a.wave_lds_floats + (SOFT ? a.N : 0u);
    float* alpha = smem + wv * per_wave; // alpha[s] at alpha + (1 << s)
    uint32_t* bits = reinterpret_cast<uint32_t*>(alpha + a.N);
    float* sw = SOFT ? smem + wv * per_wave + a.wave_lds_floats : nullptr;
    const float* y = a.llr + frame * a.N;
    const uint32_t top = a.log2N;

    for (uint32_t k = 0; k < a.nops; ++k) {
        const uint32_t w = ld_const(a.ops, k);
        const uint32_t code = op_code(w), s = op_stage(w), o = op_off(w);
        const uint64_t t0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
        if (code >= OP_L_R0) {
            if (s == top)
                sc_leaf<SOFT>(code, y, 1u << s, o, bits, lane, sw);
            else
                sc_leaf<SOFT>(code, alpha + (1u << s), 1u << s, o, bits, lane, sw);
        } else if (code == OP_COMB || code == OP_COPY0) {
            sc_bits_op(code, s, o, bits, lane);
            if constexpr (SOFT)
                soft_bits_op(code, s, o, sw, lane);
        } else {
            if (s == top)
                sc_inner<SOFT>(code, y, s, o, alpha, bits, lane, sw);
            else
                sc_inner<SOFT>(code, alpha + (1u << s), s, o, alpha, bits, lane, sw);
        }
        wsync();
        if (a.prof) {
            const uint64_t t1 = __builtin_amdgcn_s_memtime();
            if (lane == 0) {
                atomicAdd(&a.prof[2 * code], (unsigned long long)(t1 - t0));
                atomicAdd(&a.prof[2 * code + 1], 1ull);
            }
        }
    }
    if constexpr (SOFT) {
        float* out = a.soft + frame * a.N;
        for (uint32_t i = lane; i < a.N; i += 64)
            out[i] = sw[i];
    }
    if (!a.systematic)
        polar_transform_bits(bits, a.N, lane);
    const uint32_t syn = emit_info(bits, a, frame, lane, true);
    if (lane == 0 && a.ok)
        a.ok[frame] = syn == 0 ? 1 : 0;
}

template <bool SOFT>
static int launch_sc_impl(const KernelArgs& a, hipStream_t stream)
{
    const size_t per_wave = ((size_t)a.wave_lds_floats + (SOFT ? a.N : 0u)) * sizeof(float);
    if (per_wave > 160 * 1024)
        return -4;
    if (per_wave * 4 <= 160 * 1024) {
        const uint64_t blocks = (a.F + 3) / 4;
        if (blocks == 0)
            return 0;
        hipLaunchKernelGGL((sc_kernel<4, SOFT>), dim3((uint32_t)blocks), dim3(256), 4 * per_wave, stream, a);
    } else {
        if (a.F == 0)
            return 0;
        hipLaunchKernelGGL((sc_kernel<1, SOFT>), dim3((uint32_t)a.F), dim3(64), per_wave, stream, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_sc(const KernelArgs& a, hipStream_t stream)
{
    return a.soft ? launch_sc_impl<true>(a, stream) : launch_sc_impl<false>(a, stream);
}

// LDS bytes one codeword of the soft-output decode needs (0 if it does not fit a CU)
uint32_t sc_soft_lds_bytes(uint32_t N)
{
    const size_t b = ((size_t)sc_wave_lds_floats(N) + N) * sizeof(float);
    return b > 160 * 1024 ? 0u : (uint32_t)b;
}

} // namespace pcg
