// frames_kernel.hip -- the data formats either side of the decoder (SURVEY.md §8f rows
// 1-2), batched on the device:
//
//   depuncture / puncture   Puncturer::depuncture / puncture / puncturePacked
//                           (include/polarcode/puncturer.h:71-99, puncturer.cpp:71-89)
//   encode                  Detector::generate + ButterflyFipPacked::encode
//                           (butterfly_fip_packed.cpp:45-70), systematic double transform
//   random info, BPSK-AWGN  the simulator's frame source (simulator.cpp:850-937,
//                           bpsk.cpp:54-80, awgn.cpp:38-43) with a counter-based RNG
//
// All of it is byte/bit work bounded by HBM: one wave per frame for the encoder
// (packed 32-bit words, butterflies as shifts inside a word and shuffles across lanes),
// flat grid-stride float4 streams for the (de)puncturers and the channel.
#include "frames.hpp"
#include "wave.hpp"

#include <hip/hip_runtime.h>

namespace pcg {

namespace {

constexpr int kBlock = 256;

uint32_t grid_for(uint64_t items, uint32_t per_block)
{
    uint64_t g = (items + per_block - 1) / per_block;
    if (g > 65536u * 8u)
        g = 65536u * 8u; // grid-stride beyond this: ~2 k workgroups per XCD
    return (uint32_t)(g ? g : 1);
}

// ---- depuncture: out[f][n] = src[n] >= 0 ? in[f][src[n]] : +0.0f --------------------------
// (puncturer.h:92-99: fill with 0, then scatter).  Written as a gather over the output so
// every output float4 is one coalesced store; `src` (N ints) stays in L1/L2.
__global__ void __launch_bounds__(kBlock) depuncture_kernel(const float* __restrict__ in,
                                                            uint64_t F,
                                                            uint32_t E,
                                                            uint32_t N,
                                                            const int32_t* __restrict__ src,
                                                            float* __restrict__ out)
{
    const uint32_t q = N >> 2; // float4 per frame
    const uint64_t total = F * q;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t f = t / q;
        const uint32_t n = (uint32_t)(t - f * q) << 2;
        const float* row = in + f * E;
        const int4 s = *reinterpret_cast<const int4*>(src + n);
        float4 v;
        v.x = s.x >= 0 ? row[s.x] : 0.0f;
        v.y = s.y >= 0 ? row[s.y] : 0.0f;
        v.z = s.z >= 0 ? row[s.z] : 0.0f;
        v.w = s.w >= 0 ? row[s.w] : 0.0f;
        *reinterpret_cast<float4*>(out + f * N + n) = v;
    }
}

// ---- puncture: out[f][k] = in[f][pos[k]] (puncturer.h:60-67) -------------------------------
__global__ void __launch_bounds__(kBlock) puncture_kernel(const float* __restrict__ in,
                                                          uint64_t F,
                                                          uint32_t N,
                                                          uint32_t E,
                                                          const uint32_t* __restrict__ pos,
                                                          float* __restrict__ out)
{
    const uint64_t total = F * E;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t f = t / E;
        const uint32_t k = (uint32_t)(t - f * E);
        out[t] = in[f * N + pos[k]];
    }
}

// ---- puncturePacked: MSB-first bytes (puncturer.cpp:71-89); one thread per output byte ----
__global__ void __launch_bounds__(kBlock) puncture_packed_kernel(const uint8_t* __restrict__ in,
                                                                 uint64_t F,
                                                                 uint32_t N,
                                                                 uint32_t E,
                                                                 const uint32_t* __restrict__ pos,
                                                                 uint8_t* __restrict__ out)
{
    const uint32_t eb = E >> 3, nb = N >> 3;
    const uint64_t total = F * eb;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t f = t / eb;
        const uint32_t b = (uint32_t)(t - f * eb);
        const uint8_t* row = in + f * nb;
        uint32_t o = 0;
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t p = pos[8 * b + i];
            o |= ((uint32_t)(row[p >> 3] >> (7 - (p & 7))) & 1u) << (7 - i);
        }
        out[t] = (uint8_t)o;
    }
}

// ---- encoder -----------------------------------------------------------------------------
// Word layout inside the kernel: codeword position i is bit (i & 31) of word i >> 5
// (LSB-first).  The polar transform x[i] ^= x[i + B] for every B (butterfly_fip.cpp:15-63;
// the stages commute) is, for B < 32, x ^= (x >> B) & lowmask(B) inside each word, and for
// B >= 32 a XOR with the word B/32 further on.  Words live in registers: lane l holds words
// l + 64 m (m < WPL), so word distances < 64 are lane shuffles, >= 64 register moves.
__device__ __forceinline__ uint32_t lowmask(uint32_t B)
{
    // bits i with (i & B) == 0, i < 32
    switch (B) {
    case 1: return 0x55555555u;
    case 2: return 0x33333333u;
    case 4: return 0x0F0F0F0Fu;
    case 8: return 0x00FF00FFu;
    default: return 0x0000FFFFu;
    }
}

template <int WPL>
__device__ __forceinline__ void polar_transform_words(uint32_t (&w)[WPL], uint32_t nwords, uint32_t lane)
{
#pragma unroll
    for (int m = 0; m < WPL; ++m)
        for (uint32_t B = 1; B < 32; B <<= 1)
            w[m] ^= (w[m] >> B) & lowmask(B);
    for (uint32_t d = 1; d < nwords && d < 64; d <<= 1) {
#pragma unroll
        for (int m = 0; m < WPL; ++m) {
            const uint32_t up = __shfl_down(w[m], d, 64);
            if ((lane & d) == 0)
                w[m] ^= up;
        }
    }
#pragma unroll
    for (int dm = 1; dm < WPL; dm <<= 1) {
#pragma unroll
        for (int m = 0; m < WPL; ++m)
            if ((m & dm) == 0 && m + dm < WPL)
                w[m] ^= w[m + dm];
    }
}

// One wave per frame.  info (F x kb) gets the detector's check bits written in place, as
// Encoder::encode_vector does to the caller's buffer (butterfly_fip_packed.cpp:47-48).
template <int WPL>
__global__ void __launch_bounds__(256) encode_kernel(EncodeArgs a)
{
    const uint32_t lane = lane_id();
    const uint64_t frame = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (frame >= a.F)
        return;
    uint8_t* info = a.info + frame * a.kb;
    // 1) check bits: trailer = g0 ^ XOR_{j : m_j = 1} delta_j (the generate() model built
    //    and self-checked on the host, frames.cpp)
    uint32_t acc = 0;
    if (a.ntrail) {
        for (uint32_t j = lane; j < a.K; j += 64)
            if ((info[j >> 3] >> (7 - (j & 7))) & 1u)
                acc ^= a.delta[j];
        acc = wave_xor(acc) ^ a.g0;
    }
    // 2) u: info bit j at position info_pos[j]; word-wise gather through `rank`
    uint32_t w[WPL];
#pragma unroll
    for (int m = 0; m < WPL; ++m) {
        const uint32_t wi = lane + 64u * m;
        uint32_t v = 0;
        if (wi < a.nwords) {
            for (uint32_t b = 0; b < 32 && 32 * wi + b < a.N; ++b) {
                const uint32_t j = a.rank[32 * wi + b];
                if (j != 0xFFFFu)
                    v |= ((uint32_t)(info[j >> 3] >> (7 - (j & 7))) & 1u) << b;
            }
        }
        w[m] = v;
    }
    // the check bits replace what the message held there (<= 32 positions, uniform loop)
    for (uint32_t t = 0; t < a.ntrail; ++t) {
        const uint32_t p = a.info_pos[a.trail[t]];
        const uint32_t bit = (acc >> t) & 1u;
#pragma unroll
        for (int m = 0; m < WPL; ++m)
            if (lane + 64u * m == (p >> 5))
                w[m] = (w[m] & ~(1u << (p & 31))) | (bit << (p & 31));
    }
    // ... and go back into the caller's info buffer (encode_vector modifies it too)
    if (lane == 0) {
        for (uint32_t t = 0; t < a.ntrail; ++t) {
            const uint32_t j = a.trail[t];
            const uint8_t mk = (uint8_t)(0x80u >> (j & 7));
            info[j >> 3] = ((acc >> t) & 1u) ? (uint8_t)(info[j >> 3] | mk) : (uint8_t)(info[j >> 3] & ~mk);
        }
    }
    polar_transform_words<WPL>(w, a.nwords, lane);
    if (a.systematic) {
#pragma unroll
        for (int m = 0; m < WPL; ++m) {
            const uint32_t wi = lane + 64u * m;
            if (wi < a.nwords)
                w[m] &= a.infomask[wi];
        }
        polar_transform_words<WPL>(w, a.nwords, lane);
    }
    // 3) MSB-first bytes (PackedContainer layout, bitcontainer.cpp:975-992)
    uint8_t* code = a.code + frame * (a.N >> 3);
#pragma unroll
    for (int m = 0; m < WPL; ++m) {
        const uint32_t wi = lane + 64u * m;
        if (wi < a.nwords) {
            const uint32_t r = __builtin_bitreverse32(w[m]); // position 32wi+b -> bit 31-b
            if (a.N >= 32) {
                // bytes 4wi..4wi+3: byte k = positions 8k..8k+7, position 8k at the MSB
                const uint32_t be = __builtin_bswap32(r);
                *reinterpret_cast<uint32_t*>(code + 4 * wi) = be;
            } else {
                for (uint32_t k = 0; k < (a.N >> 3); ++k)
                    code[k] = (uint8_t)(r >> (24 - 8 * k));
            }
        }
    }
}

// ---- counter-based RNG: Philox4x32-10 (Salmon et al., SC'11) ---------------------------
struct U4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
        const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        c = U4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// uniform info bytes; the bits past K in the last byte are cleared
__global__ void __launch_bounds__(kBlock) random_info_kernel(uint8_t* __restrict__ info,
                                                            uint64_t F,
                                                            uint32_t kb,
                                                            uint32_t K,
                                                            uint64_t seed)
{
    const uint32_t q = (kb + 15) / 16; // 16 bytes per Philox call
    const uint64_t total = F * q;
    const uint8_t tailmask = (K & 7) ? (uint8_t)(0xFFu << (8 - (K & 7))) : 0xFFu;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t f = t / q;
        const uint32_t c = (uint32_t)(t - f * q);
        const U4 r = philox(U4{c, (uint32_t)f, (uint32_t)(f >> 32), 0x1F0u}, (uint32_t)seed, (uint32_t)(seed >> 32));
        const uint32_t words[4] = {r.x, r.y, r.z, r.w};
        uint8_t* row = info + f * kb;
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            const uint32_t idx = 16 * c + b;
            if (idx < kb) {
                uint8_t v = (uint8_t)(words[b >> 2] >> (8 * (b & 3)));
                if (idx == kb - 1)
                    v &= tailmask;
                row[idx] = v;
            }
        }
    }
}

// BPSK (bit 0 -> +1, bpsk.cpp:54-80) + AWGN + LLR = 2 y / sigma^2 (simulator.cpp:832-838).
// Thread t makes 4 consecutive symbols from one Philox call (Box-Muller twice).
__global__ void __launch_bounds__(kBlock) bpsk_awgn_kernel(const uint8_t* __restrict__ code,
                                                          uint64_t F,
                                                          uint32_t n,
                                                          float sigma,
                                                          uint64_t seed,
                                                          float* __restrict__ llr)
{
    const uint32_t q = n >> 2;
    const uint64_t total = F * q;
    const float scale = sigma > 0.0f ? 2.0f / (sigma * sigma) : 1.0f;
    const uint32_t nb = n >> 3;
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t f = t / q;
        const uint32_t i = (uint32_t)(t - f * q) << 2;
        const uint8_t byte = code[f * nb + (i >> 3)];
        float s[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            s[k] = ((byte >> (7 - ((i + k) & 7))) & 1u) ? -1.0f : 1.0f;
        if (sigma > 0.0f) {
            const U4 r = philox(U4{i, (uint32_t)f, (uint32_t)(f >> 32), 0xA96u}, (uint32_t)seed, (uint32_t)(seed >> 32));
            const float u1a = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f); // (0, 1]
            const float u2a = (float)(r.y >> 8) * (1.0f / 16777216.0f);          // [0, 1)
            const float u1b = ((float)(r.z >> 8) + 1.0f) * (1.0f / 16777216.0f);
            const float u2b = (float)(r.w >> 8) * (1.0f / 16777216.0f);
            const float ra = sqrtf(-2.0f * logf(u1a)), rb = sqrtf(-2.0f * logf(u1b));
            float sa, ca, sb, cb;
            sincospif(2.0f * u2a, &sa, &ca);
            sincospif(2.0f * u2b, &sb, &cb);
            s[0] += sigma * ra * ca;
            s[1] += sigma * ra * sa;
            s[2] += sigma * rb * cb;
            s[3] += sigma * rb * sb;
        }
        *reinterpret_cast<float4*>(llr + f * n + i) =
            make_float4(scale * s[0], scale * s[1], scale * s[2], scale * s[3]);
    }
}

// ---- adaptive decoding: the frames whose first-stage check failed ---------------------------
// fmap[0 .. *count) = { f : ok[f] == 0 } (any order; *count zeroed by the caller).  One atomic
// per wave: ballot, popcount, lane-prefix.
__global__ void __launch_bounds__(kBlock) compact_failed_kernel(const uint8_t* __restrict__ ok,
                                                               uint64_t F,
                                                               uint32_t* __restrict__ fmap,
                                                               uint32_t* __restrict__ count)
{
    const uint32_t lane = lane_id();
    for (uint64_t base = ((uint64_t)blockIdx.x * kBlock + (threadIdx.x & ~63u)); base < F;
         base += (uint64_t)gridDim.x * kBlock) {
        const uint64_t f = base + lane;
        const bool fail = f < F && ok[f] == 0;
        const uint64_t m = ballot(fail);
        if (m == 0)
            continue;
        uint32_t off = 0;
        if (lane == 0)
            off = atomicAdd(count, (uint32_t)__builtin_popcountll(m));
        off = __shfl(off, 0, 64);
        if (fail)
            fmap[off + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull))] = (uint32_t)f;
    }
}

} // namespace

int launch_compact_failed(const uint8_t* ok, uint64_t F, uint32_t* fmap, uint32_t* count, hipStream_t s)
{
    if (hipMemsetAsync(count, 0, sizeof(uint32_t), s) != hipSuccess)
        return -3;
    if (F == 0)
        return 0;
    hipLaunchKernelGGL(compact_failed_kernel, dim3(grid_for(F, kBlock)), dim3(kBlock), 0, s, ok, F, fmap, count);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_depuncture(const float* in, uint64_t F, uint32_t E, uint32_t N, const int32_t* src, float* out,
                      hipStream_t s)
{
    if (F == 0)
        return 0;
    hipLaunchKernelGGL(depuncture_kernel, dim3(grid_for(F * (N / 4), kBlock)), dim3(kBlock), 0, s, in, F, E, N, src,
                       out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_puncture(const float* in, uint64_t F, uint32_t N, uint32_t E, const uint32_t* pos, float* out,
                    hipStream_t s)
{
    if (F == 0)
        return 0;
    hipLaunchKernelGGL(puncture_kernel, dim3(grid_for(F * E, kBlock)), dim3(kBlock), 0, s, in, F, N, E, pos, out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_puncture_packed(const uint8_t* in, uint64_t F, uint32_t N, uint32_t E, const uint32_t* pos, uint8_t* out,
                           hipStream_t s)
{
    if (F == 0)
        return 0;
    hipLaunchKernelGGL(puncture_packed_kernel, dim3(grid_for(F * (E / 8), kBlock)), dim3(kBlock), 0, s, in, F, N, E,
                       pos, out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_encode(const EncodeArgs& a, hipStream_t s)
{
    if (a.F == 0)
        return 0;
    const dim3 grid((uint32_t)((a.F + 3) / 4)), block(256);
    const uint32_t wpl = (a.nwords + 63) / 64;
    if (wpl <= 1)
        hipLaunchKernelGGL(encode_kernel<1>, grid, block, 0, s, a);
    else if (wpl <= 2)
        hipLaunchKernelGGL(encode_kernel<2>, grid, block, 0, s, a);
    else if (wpl <= 4)
        hipLaunchKernelGGL(encode_kernel<4>, grid, block, 0, s, a);
    else if (wpl <= 8)
        hipLaunchKernelGGL(encode_kernel<8>, grid, block, 0, s, a);
    else if (wpl <= 16)
        hipLaunchKernelGGL(encode_kernel<16>, grid, block, 0, s, a);
    else
        return -4;
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_random_info(uint8_t* info, uint64_t F, uint32_t K, uint64_t seed, hipStream_t s)
{
    const uint32_t kb = (K + 7) / 8;
    if (F == 0 || kb == 0)
        return 0;
    hipLaunchKernelGGL(random_info_kernel, dim3(grid_for(F * ((kb + 15) / 16), kBlock)), dim3(kBlock), 0, s, info, F,
                       kb, K, seed);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_bpsk_awgn(const uint8_t* code, uint64_t F, uint32_t n, float sigma, uint64_t seed, float* llr,
                     hipStream_t s)
{
    if (F == 0)
        return 0;
    hipLaunchKernelGGL(bpsk_awgn_kernel, dim3(grid_for(F * (n / 4), kBlock)), dim3(kBlock), 0, s, code, F, n, sigma,
                       seed, llr);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

} // namespace pcg
