// crc_host.hpp -- host implementations of the reference's error detectors.
//
// Shared by the plan builder (to derive the affine GF(2) syndrome tables the GPU
// kernels use) and by the host Detector classes (include/polarcode/errordetection).
//   CRC8   src/polarcode/errordetection/crc8.cpp:18-57   poly 0x07, init 0, last byte
//   CRC16  src/polarcode/errordetection/crc16.cpp:21-43  CCITT-FALSE via CRC++ (CRC.h),
//                                                        big-endian in the last 2 bytes
//   CRC32  src/polarcode/errordetection/crc32.cpp:28-66  CRC-32C (_mm_crc32_u32) over
//                                                        little-endian words, init 0
//   CRC11  not in the reference: 3GPP TS 38.212 §5.1 gCRC11(D) =
//          D^11+D^10+D^9+D^5+1, init 0, over the bit stream of the message
//          (MSB-first bytes); the 11 parity bits occupy the last 11 bits, MSB first.
#pragma once
#include <cstdint>
#include <cstring>

namespace pcg {

inline uint8_t crc8_gen(const uint8_t* d, int bytes)
{
    uint8_t c = 0;
    for (int i = 0; i < bytes; ++i) {
        c ^= d[i];
        for (int b = 0; b < 8; ++b)
            c = (uint8_t)((c << 1) ^ ((c & 0x80) ? 0x07 : 0));
    }
    return c;
}

inline uint16_t crc16_gen(const uint8_t* d, int bytes)
{
    uint16_t c = 0xFFFF;
    for (int i = 0; i < bytes; ++i) {
        c ^= (uint16_t)(d[i] << 8);
        for (int b = 0; b < 8; ++b)
            c = (uint16_t)((c & 0x8000) ? (c << 1) ^ 0x1021 : (c << 1));
    }
    return c;
}

inline uint32_t crc32c_gen(const uint8_t* d, int words)
{
    uint32_t c = 0;
    for (int w = 0; w < words; ++w) {
        uint32_t v;
        std::memcpy(&v, d + 4 * w, 4); // little-endian host
        c ^= v;
        for (int b = 0; b < 32; ++b)
            c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    }
    return c;
}

// remainder of m(D)*D^11 mod gCRC11 over the first `nbits` bits of d (MSB-first)
inline uint32_t crc11_gen(const uint8_t* d, int nbits)
{
    uint32_t c = 0;
    for (int i = 0; i < nbits; ++i) {
        const uint32_t fb = ((c >> 10) ^ (uint32_t)(d[i >> 3] >> (7 - (i & 7)))) & 1u;
        c = (c << 1) & 0x7FFu;
        if (fb)
            c ^= 0x621u;
    }
    return c;
}

// the trailing 11 bits of a `bytes`-byte message
inline uint32_t crc11_tail(const uint8_t* d, int bytes)
{
    uint32_t t = 0;
    for (int i = bytes * 8 - 11; i < bytes * 8; ++i)
        t = (t << 1) | ((uint32_t)(d[i >> 3] >> (7 - (i & 7))) & 1u);
    return t;
}

// Syndrome of the detector over a message of `bytes` bytes: zero <=> check() passes.
// kind: 0 (Dummy, always 0), 8, 11, 16, 32.  Returns false for an unknown kind.
inline bool crc_syndrome(int kind, const uint8_t* d, int bytes, uint32_t* syn)
{
    switch (kind) {
    case 0:
        *syn = 0;
        return true;
    case 8:
        *syn = bytes >= 1 ? (uint32_t)(crc8_gen(d, bytes - 1) ^ d[bytes - 1]) : 0u;
        return true;
    case 16:
        if (bytes < 2) { *syn = 0; return true; }
        *syn = (uint32_t)(crc16_gen(d, bytes - 2) ^
                          (uint16_t)((d[bytes - 2] << 8) | d[bytes - 1]));
        return true;
    case 11:
        *syn = bytes >= 2 ? crc11_gen(d, bytes * 8 - 11) ^ crc11_tail(d, bytes) : 0u;
        return true;
    case 32: {
        int rw = (bytes >> 2) - 1;
        if (rw < 0) { *syn = 0; return true; }
        uint32_t s;
        std::memcpy(&s, d + 4 * rw, 4);
        *syn = crc32c_gen(d, rw) ^ s;
        return true;
    }
    default:
        return false;
    }
}

inline bool crc_check(int kind, const uint8_t* d, int bytes)
{
    uint32_t s = 1;
    return crc_syndrome(kind, d, bytes, &s) && s == 0;
}

// Detector::generate: write the checksum into the trailing byte(s)/word.
inline bool crc_generate(int kind, uint8_t* d, int bytes)
{
    switch (kind) {
    case 0:
        return true;
    case 8:
        d[bytes - 1] = crc8_gen(d, bytes - 1);
        return true;
    case 16: {
        uint16_t c = crc16_gen(d, bytes - 2);
        d[bytes - 2] = (uint8_t)(c >> 8);
        d[bytes - 1] = (uint8_t)c;
        return true;
    }
    case 11: {
        if (bytes < 2)
            return true;
        const uint32_t c = crc11_gen(d, bytes * 8 - 11);
        for (int k = 0; k < 11; ++k) {
            const int i = bytes * 8 - 11 + k;
            const uint8_t m = (uint8_t)(0x80u >> (i & 7));
            d[i >> 3] = (uint8_t)(((c >> (10 - k)) & 1u) ? (d[i >> 3] | m) : (d[i >> 3] & ~m));
        }
        return true;
    }
    case 32: {
        int rw = (bytes / 4) - 1;
        std::memset(d + 4 * rw, 0, 4);
        uint32_t c = crc32c_gen(d, rw);
        std::memcpy(d + 4 * rw, &c, 4);
        return true;
    }
    default:
        return false;
    }
}

} // namespace pcg
