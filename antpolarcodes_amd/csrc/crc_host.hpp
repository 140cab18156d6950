// crc_host.hpp -- host implementations of the reference's error detectors.
//
// Shared by the plan builder (to derive the affine GF(2) syndrome tables the GPU
// kernels use) and by the host Detector classes (include/polarcode/errordetection).
//   CRC8   src/polarcode/errordetection/crc8.cpp:18-57   poly 0x07, init 0, last byte
//   CRC16  src/polarcode/errordetection/crc16.cpp:21-43  CCITT-FALSE via CRC++ (CRC.h),
//                                                        big-endian in the last 2 bytes
//   CRC32  src/polarcode/errordetection/crc32.cpp:28-66  CRC-32C (_mm_crc32_u32) over
//                                                        little-endian words, init 0
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

// Syndrome of the detector over a message of `bytes` bytes: zero <=> check() passes.
// kind: 0 (Dummy, always 0), 8, 16, 32.  Returns false for an unknown kind.
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
