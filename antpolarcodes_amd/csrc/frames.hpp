// frames.hpp -- device launch interface of frames_kernel.hip (puncturer, encoder,
// frame source) and the C-ABI objects built on it (frames_capi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace pcg {

struct EncodeArgs {
    uint64_t F;
    uint32_t N, K, kb, nwords;
    uint8_t* info;             // F x kb (device), check bits written in place
    uint8_t* code;             // F x N/8 (device), MSB-first packed codeword
    const uint16_t* rank;      // N: info-bit index at codeword position, 0xFFFF if frozen
    const uint16_t* info_pos;  // K: codeword position of info bit j
    const uint32_t* infomask;  // nwords: 1 at non-frozen positions (LSB-first words)
    int systematic;
    uint32_t ntrail;           // check bits the detector writes (<= 32)
    const uint16_t* trail;     // ntrail info-bit indices they occupy
    const uint32_t* delta;     // K: trailer flips caused by info bit j
    uint32_t g0;               // trailer of the all-zero message
};

int launch_depuncture(const float* in, uint64_t F, uint32_t E, uint32_t N, const int32_t* src, float* out,
                      hipStream_t s);
int launch_puncture(const float* in, uint64_t F, uint32_t N, uint32_t E, const uint32_t* pos, float* out,
                    hipStream_t s);
int launch_puncture_packed(const uint8_t* in, uint64_t F, uint32_t N, uint32_t E, const uint32_t* pos, uint8_t* out,
                           hipStream_t s);
int launch_encode(const EncodeArgs& a, hipStream_t s);
// adaptive decoding: indices of frames with ok == 0 into fmap, their number into *count
int launch_compact_failed(const uint8_t* ok, uint64_t F, uint32_t* fmap, uint32_t* count, hipStream_t s);
int launch_random_info(uint8_t* info, uint64_t F, uint32_t K, uint64_t seed, hipStream_t s);
int launch_bpsk_awgn(const uint8_t* code, uint64_t F, uint32_t n, float sigma, uint64_t seed, float* llr,
                     hipStream_t s);

// Puncturer(E, frozen) (puncturer.cpp:51-66) on the host: parent length and kept positions.
// Returns 0, or -1 with *err set (the reference's std::out_of_range text).
int build_puncturer(uint32_t E, const uint32_t* frozen, uint32_t nf, uint32_t* N, std::vector<uint32_t>* pos,
                    const char** err);

} // namespace pcg

// the C-ABI puncturer object (include/pcg.h), shared with capi.cpp's punctured decode
struct pcg_puncturer {
    uint32_t E = 0, N = 0;
    int device = -1;
    std::vector<uint32_t> pos; // host copy of the kept parent positions
    uint32_t* d_pos = nullptr; // E
    int32_t* d_src = nullptr;  // N: source index in the punctured frame or -1
};
