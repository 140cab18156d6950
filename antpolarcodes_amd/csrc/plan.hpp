// plan.hpp -- decoder plan: the reference's decoder tree, classified exactly as the
// reference does, flattened into a wave-uniform op schedule for the HIP kernels.
//
// Fast-SSC classification : FastSscAvx::createDecoder, fastssc_avx_float.cpp:797-896
// SCL classification      : SclAvx::createDecoder,     scl_avx_float.cpp:624-651
// frozen-set split        : splitFrozenBits,           src/polarcode/polarcode.cpp:14-34
#pragma once
#include <cstdint>
#ifndef PCG_RTC // (plan-specialised kernels compile the device part of this header with hiprtc)
#include <string>
#include <vector>
#endif

#if defined(__HIPCC__) || defined(__HIP__)
#define PCG_HD __host__ __device__
#else
#define PCG_HD
#endif

namespace pcg {

// One op = one 32-bit word: code | stage << 8 | offset << 16.
//   stage  = log2 of the node size n (the op reads alpha[stage], for F/G writes
//            alpha[stage-1]);  offset = first codeword-bit position of the node.
enum OpCode : uint32_t {
    // internal-node ops (Fast-SSC and SCL)
    OP_F = 1,     // alpha[s-1][i] = f(alpha[s][i], alpha[s][i+h])            avx_float.h:101-127
    OP_G = 2,     // alpha[s-1][i] = g(alpha[s][i], alpha[s][i+h], bit[o+i])  avx_float.h:147-164
    OP_G0 = 3,    // alpha[s-1][i] = alpha[s][i] + alpha[s][i+h]   (ZeroRNode) avx_float.h:166-175
    OP_COMB = 4,  // bit[o+i] ^= bit[o+h+i]                                    avx_float.h:188-197
    OP_COPY0 = 5, // bit[o+i]  = bit[o+h+i]                        (ZeroRNode) avx_float.h:199-204
    OP_RONE = 6,  // fused right rate-1 of ROneNode             fastssc_avx_float.cpp:205-219
    // Fast-SSC leaves (fastssc_avx_float.cpp)
    OP_L_R0 = 16,    // :247
    OP_L_R1 = 17,    // :257-263
    OP_L_REP = 18,   // :273-287
    OP_L_SPC = 19,   // :342-373
    OP_L_DREP = 20,  // :303-332
    OP_L_DSPC = 21,  // :425-466
    OP_L_DSPC8 = 22, // :473-488
    OP_L_TREP = 23,  // :572-589
    OP_L_TYPE5 = 24, // :762-792
    OP_L_REPR1 = 25, // :718-739
    OP_L_ZSPC8 = 26, // :556-565
    OP_L_ZSPC = 27,  // :503-546 (reproduces the reference's right-half output, Q1)
    // scq_kernel.hip only (PlanHost::ops_fused): a size-16 RateRNode whose children are size-8
    // leaves (F, leaf, G, leaf, COMB) or a size-16 ROneNode over a size-8 leaf (F, leaf,
    // RONE), run in registers as one op; the next word holds the leaf codes (left | right << 8).
    // In ops_fused the stage byte also carries, in its high nibble, the number of parent
    // COMB levels folded into the op (plan.cpp fuse_sc16).
    OP_Q16 = 28,
    OP_Q16R = 29,
    // ... preceded by its parent's F (left child: OP_Q16F) or G (right child: OP_Q16G) from the
    // size-32 stage; offset = the size-16 child's; descriptor bit 16 = the child is a Q16R,
    // bit 17 = the child is a size-16 leaf whose code is the descriptor's low byte
    OP_Q16F = 30,
    OP_Q16G = 31,
    // SCL leaves (scl_avx_float.cpp)
    OP_S_R0 = 40,  // :316-337
    OP_S_R1 = 41,  // :353-413
    OP_S_REP = 42, // :428-481
    OP_S_SPC = 43, // :498-621
    // A whole size-8 SCL subtree run lane-serially (lane = path) in registers; the
    // next schedule word is its descriptor (see scl_emit in plan.cpp).
    OP_S_ST8 = 44,
    // 8-bit fixed-point Fast-SSC leaves (FastSscFipChar, fastssc_fip_char.cpp); the
    // internal ops above (F, G, G0, RONE, COMB, COPY0) take the char semantics of
    // fip_char.h in the int8 kernels
    OP_C_R0 = 64,    // RateZeroDecoder            :202-208
    OP_C_R1 = 65,    // RateOneDecoder             :210-215
    OP_C_REP = 66,   // RepetitionDecoder, n > 32  :225-241
    OP_C_REPS = 67,  // ShortRepetitionDecoder     :265-272
    OP_C_DREP = 68,  // DoubleRepetitionDecoder    :249-263
    OP_C_SPC = 69,   // SpcDecoder, n > 32         :274-303
    OP_C_SPCS = 70,  // ShortSpcDecoder            :305-319
    OP_C_ZSPC = 71,  // ZeroSpcDecoder, n > 32     :321-359
    OP_C_ZSPCS = 72, // ShortZeroSpcDecoder        :361-388
    OP_C_ZONES = 73, // ShortZeroOneDecoder        :390-399
    // 8-bit fixed-point SCL leaves (SclFipChar, scl_fip_char.cpp)
    OP_CS_R0 = 80,  // RateZeroDecoder   :387-421
    OP_CS_R1 = 81,  // RateOneDecoder    :423-505
    OP_CS_REP = 82, // RepetitionDecoder :508-580
    OP_CS_SPC = 83, // SpcDecoder        :583-726
};

// ST8 descriptor: per size-4 child c (c = 0 left, 1 right) at bits 8c..8c+6:
// [0..2] kind (ST_R0, ST_R1, ST_REP, ST_SPC, ST_RATER), [3..4] / [5..6] kinds of its
// size-2 children when it is a RateR (ST_R0, ST_R1, ST_REP).
enum StKind : uint32_t { ST_R0 = 0, ST_R1 = 1, ST_REP = 2, ST_SPC = 3, ST_RATER = 4 };

constexpr PCG_HD inline uint32_t op_code(uint32_t w) { return w & 0xffu; }
constexpr PCG_HD inline uint32_t op_stage(uint32_t w) { return (w >> 8) & 0xffu; }
constexpr PCG_HD inline uint32_t op_off(uint32_t w) { return w >> 16; }
// ops of the fused schedule followed by a descriptor word
constexpr PCG_HD inline bool op_has_desc(uint32_t code) { return code >= 28 && code <= 31; }

#ifndef PCG_RTC
struct PlanHost {
    uint32_t N = 0, K = 0, L = 1, log2N = 0;
    int systematic = 1;
    int crc_kind = 0;
    std::vector<uint32_t> frozen;
    std::vector<uint32_t> ops;      // flattened schedule
    std::vector<uint32_t> ops_fused; // Fast-SSC float: `ops` with size-16 leaf pairs fused (OP_Q16/Q16R)
    std::vector<uint16_t> info_pos; // K non-frozen positions, ascending (bitcontainer.cpp:68-84)
    std::vector<uint32_t> crc_m;    // K affine syndrome columns
    uint32_t crc_c0 = 0;            // syndrome of the all-zero message
    std::vector<uint32_t> crc_rows; // crc_kind x W codeword-position masks of the same model
    uint32_t node_count = 0;
    std::vector<int> node_types;    // pre-order census (op code of each node; 0 = internal)
    bool scl_st8 = true;            // emit lane-serial size-8 subtrees for SCL
    int fixed = 0;                  // 1: the reference's 8-bit decoders (FastSscFipChar / SclFipChar)
    int sc_kind = 0;  // Fast-SSC kernel: 2 = scq (LDS-resident), 0 = lane-serial, 1 = one codeword per wave
    uint32_t scq_q = 16; // scq: lanes per codeword
    int scq_virt = 1;     // scq: the root's children recomputed from the channel
};

// Returns 0, or a negative pcg.h error code with *err set.
int build_plan(PlanHost& p,
               uint32_t N,
               uint32_t L,
               const uint32_t* frozen,
               uint32_t nf,
               int systematic,
               int crc_kind,
               std::string* err,
               int fixed = 0);
#endif

} // namespace pcg
