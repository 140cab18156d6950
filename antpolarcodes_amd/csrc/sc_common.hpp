// sc_common.hpp -- packed-codeword-bit helpers shared by the one-codeword-per-wave
// Fast-SSC kernels (sc_kernel.hip: float, sc_char_kernel.hip: int8) and the SCL kernels.
#pragma once
#include "kernels.hpp"
#include "plan.hpp"
#include "wave.hpp"

namespace pcg {

// fill positions [o, o+n) with one bit value
PCG_DEV void fill_bits(uint32_t* w, uint32_t o, uint32_t n, uint32_t bit, uint32_t lane)
{
    if (n >= 32) {
        const uint32_t v = bit ? 0xffffffffu : 0u;
        for (uint32_t i = lane; i < n / 32; i += 64)
            w[(o >> 5) + i] = v;
    } else if (lane == 0) {
        const uint32_t sh = o & 31, msk = ((1u << n) - 1u) << sh;
        w[o >> 5] = (w[o >> 5] & ~msk) | (bit ? msk : 0u);
    }
}

// positions [o, o+n) get bit pattern[(i) % period] (period 2, 4 or 8); `pat` bit k = value k
PCG_DEV void fill_pattern(uint32_t* w, uint32_t o, uint32_t n, uint32_t pat, uint32_t period, uint32_t lane)
{
    uint32_t word = 0;
    for (uint32_t k = 0; k < 32; ++k)
        word |= ((pat >> (k % period)) & 1u) << k;
    if (n >= 32) {
        for (uint32_t i = lane; i < n / 32; i += 64)
            w[(o >> 5) + i] = word;
    } else if (lane == 0) {
        const uint32_t sh = o & 31, msk = ((1u << n) - 1u) << sh;
        w[o >> 5] = (w[o >> 5] & ~msk) | ((word << sh) & msk);
    }
}

// COMB (bit[o+i] ^= bit[o+h+i]) / COPY0 (bit[o+i] = bit[o+h+i]) on packed bits
PCG_DEV void sc_bits_op(uint32_t code, uint32_t s, uint32_t o, uint32_t* bits, uint32_t lane)
{
    const uint32_t h = 1u << (s - 1);
    if (h >= 32) {
        const uint32_t wl = o >> 5, wr = (o + h) >> 5;
        for (uint32_t i = lane; i < h / 32; i += 64)
            bits[wl + i] = (code == OP_COMB) ? (bits[wl + i] ^ bits[wr + i]) : bits[wr + i];
    } else if (lane == 0) {
        const uint32_t sh = o & 31, msk = ((1u << h) - 1u) << sh;
        const uint32_t w = bits[o >> 5];
        const uint32_t r = (w >> h) & msk;
        bits[o >> 5] = (code == OP_COMB) ? (w ^ r) : ((w & ~msk) | r);
    }
}

// Non-systematic re-encode in place: x -> u = x G_N on the packed bits
// (ButterflyFipPacked transform, butterfly_fip.cpp:15-63).  Shared with SCL.
PCG_DEV void polar_transform_bits(uint32_t* bits, uint32_t N, uint32_t lane)
{
    const uint32_t W = N >= 32 ? N / 32 : 1;
    for (uint32_t i = lane; i < W; i += 64)
        bits[i] = transform_word(bits[i], N);
    wsync();
    for (uint32_t d = 1; d < W; d <<= 1) {
        for (uint32_t i = lane; i < W; i += 64)
            if (!(i & d))
                bits[i] ^= bits[i + d];
        wsync();
    }
}

// Gather the info bits MSB-first (getPackedInformationBits, bitcontainer.cpp:225-292),
// optionally store them, and return the detector syndrome (0 <=> check() passes).
PCG_DEV uint32_t emit_info(const uint32_t* bits, const KernelArgs& a, uint64_t frame, uint32_t lane, bool write)
{
    uint32_t syn = 0;
    for (uint32_t b = lane; b < a.kb; b += 64) {
        uint32_t byte = 0;
        for (uint32_t j = 0; j < 8; ++j) {
            const uint32_t idx = 8 * b + j;
            if (idx < a.K) {
                const uint32_t bit = get_bit(bits, a.info_pos[idx]);
                byte |= bit << (7 - j);
                if (bit)
                    syn ^= a.crc_m[idx];
            }
        }
        if (write)
            a.info[frame * a.kb + b] = (uint8_t)byte;
    }
    return wave_xor(syn) ^ a.crc_c0;
}

} // namespace pcg
