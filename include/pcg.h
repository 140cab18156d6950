/*
 * pcg.h -- C ABI of the MI355X polar-code decoder (libpcg.so).
 *
 * This is the drop-in boundary: plain pointers and sizes, no C++ or torch types.
 * The host C++ library (include/polarcode/, mirroring the reference's
 * PolarCode::Decoding::Decoder family) and the Python module (pypolar-compatible)
 * sit on top of it; any other FFI (ctypes, cgo, JNI) can bind it directly.
 *
 * Each entry point replaces a reference interface (paths relative to the
 * reference repository david13pod/antPolarCodes):
 *
 *   pcg_plan_create   <- Decoding::create / makeDecoder + Decoder::initialize,
 *                        src/polarcode/decoding/decoder.cpp:26-87,
 *                        FastSscAvxFloat::initialize fastssc_avx_float.cpp:916-938,
 *                        SclAvxFloat::initialize scl_avx_float.cpp:674-694,
 *                        Decoder::setSystematic decoder.cpp:132,
 *                        Decoder::setErrorDetection decoder.cpp:136
 *   pcg_decode_f32    <- Decoder::decode_vector(const float*, void*) decoder.cpp:154-167,
 *                        batched: F frames per call, device-resident buffers
 *   pcg_decode_f32_host <- the same with host buffers (H2D + decode + D2H)
 *   pcg_decode_f32_soft[_host] <- decode + Decoder::getSoftCodeword (decoder.cpp:147,
 *                        FloatContainer::getSoftBits bitcontainer.cpp:294-297)
 *   pcg_plan_create_adaptive <- makeDecoder(..., 2) = AdaptiveFloat, decoder.cpp:75,
 *                        adaptive_float.cpp:14-45 (SC first, SCL for the failures)
 *   pcg_plan_create_char <- Decoding::create(..., "char") / makeDecoder(..., 0): the 8-bit
 *                        FastSscFipChar (L = 1, fastssc_fip_char.cpp:573-631) and SclFipChar
 *                        (L >= 2, scl_fip_char.cpp:759-856), decoder.cpp:37-38, 62-80
 *   pcg_decode_i8     <- Decoder::decode_vector(const char*, void*) decoder.cpp:169-181,
 *                        batched, device-resident int8 LLRs
 *   pcg_decode_i8_host <- the same with host buffers
 *   pcg_plan_create_adaptive_char <- AdaptiveChar, adaptive_char.cpp:14-45
 *   pcg_plan_destroy  <- Decoder::~Decoder decoder.cpp:104-114
 *   pcg_last_error    <- the std::exception text the reference throws
 *   pcg_puncturer_*   <- PolarCode::Puncturer (include/polarcode/puncturer.h:33-99,
 *                        src/polarcode/puncturer.cpp:51-89): depuncture / puncture /
 *                        puncturePacked over F frames on the device
 *   pcg_decode_punctured_f32 <- Puncturer::depuncture + Decoder::decode_vector, fused
 *                        into one call (the 5G NR uplink chain)
 *   pcg_encoder_*, pcg_encode <- Encoding::ButterflyFipPacked + Detector::generate
 *                        (src/polarcode/encoding/butterfly_fip_packed.cpp:45-70,
 *                        encoder.cpp:79-90), F frames on the device
 *   pcg_random_info, pcg_bpsk_awgn_f32 <- the simulator's frame source
 *                        (src/simulation/simulator.cpp:850-937, bpsk.cpp:54-80,
 *                        awgn.cpp:38-43), counter-based and reproducible from a seed
 *
 *   pcg_plan_set_initial_metric <- the SCL path-metric carry of a reused decoder
 *                        instance (PathList::setFirstPath keeps mMetric[0],
 *                        scl_avx_float.cpp:31, 99-109)
 *
 * Error model: every function returns 0 on success or a negative PCG_E* code;
 * nothing throws across the ABI.  pcg_last_error() (thread-local) describes the
 * most recent failure on the calling thread.
 *
 * Threading and streams: a plan is like the reference's stateful Decoder objects (one per
 * worker thread, simulator.cpp:703-764): its scratch, work queue, staging and adaptive
 * frame-map buffers are reused by every decode call, so a plan must be used from one host
 * thread at a time.  Decodes of one plan may be issued on different streams: each decode
 * waits (hipStreamWaitEvent) for the plan's previous decode, whichever stream ran it, so
 * they never overlap; the SCL work-queue counter is zeroed on the launch stream before
 * every launch; pcg_plan_destroy waits for the plan's last decode before freeing.  Plans
 * are independent of each other: one plan per stream / per GPU runs concurrently.
 */
#ifndef PCG_H
#define PCG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PCG_OK 0
#define PCG_E_ARG (-1)         /* bad argument (sizes, null pointers, N not a power of 2) */
#define PCG_E_FROZEN (-2)      /* frozen pattern the reference rejects with std::invalid_argument
                                  (fastssc_avx_float.cpp:821-825, 839-843) */
#define PCG_E_HIP (-3)         /* HIP runtime error (allocation, launch, copy) */
#define PCG_E_UNSUPPORTED (-4) /* valid for the reference, not (yet) for this build */
#define PCG_E_NODEVICE (-5)    /* no GPU / HIP runtime unavailable */

/* Error-detection kind used to choose the SCL output path and to fill `ok`
 * (ErrorDetection::create(size, "crc"), errordetector.cpp:23-67). */
#define PCG_CRC_NONE 0  /* Dummy: check() always true (dummy.cpp:27)                 */
#define PCG_CRC8 8      /* CRC-8, poly 0x07 (crc8.cpp)                              */
#define PCG_CRC11 11    /* 3GPP TS 38.212 CRC-11 over the bit stream, parity in the
                           last 11 bits -- NOT in the reference     */
#define PCG_CRC16 16    /* CRC-16/CCITT-FALSE, big-endian trailer (crc16.cpp)       */
#define PCG_CRC32C 32   /* CRC-32C over little-endian words (crc32.cpp)             */

typedef struct pcg_plan pcg_plan;

typedef struct pcg_plan_desc {
    uint32_t block_length;  /* N */
    uint32_t info_length;   /* K = N - |frozen| */
    uint32_t list_size;     /* L (1 = Fast-SSC) */
    uint32_t node_count;    /* decoder tree nodes */
    uint32_t op_count;      /* flattened schedule length */
    uint32_t lds_bytes;     /* LDS per codeword */
    uint64_t scratch_bytes; /* global scratch per codeword */
    int32_t crc_kind;
    int32_t systematic;
    uint32_t lanes_per_codeword; /* SCL: lanes of a wave per codeword (list size rounded up, or
                                    wider); Fast-SSC scq kernel: its Q; 0 for the other kernels */
    uint32_t dev_overrides;      /* PCG_DEV_* bits: developer environment switches
                                    that changed this plan's kernel or layout; 0 in production */
    uint32_t recomputed_stages;  /* lane-serial SCL: top LLR stages recomputed from the channel
                                    where read instead of stored (1: the root's children, 2:
                                    also its grandchildren); 0 for the other kernels */
    uint32_t specialized;        /* 1: decodes run the plan-specialised kernel (pcg_plan_specialize;
                                    an adaptive plan: both of its stages) */
} pcg_plan_desc;

#define PCG_DEV_SCL_LP 0x1   /* PCG_SCL_LP / PCG_ADAPT_LP (only when the caller passed 0) */
#define PCG_DEV_SCL_FUSE 0x2 /* PCG_SCL_FUSE */
#define PCG_DEV_SCQ 0x4      /* PCG_SCQ_Q / PCG_SCQ_VIRT */
#define PCG_DEV_LAYOUT 0x8   /* PCG_SC_KERNEL, PCG_*_LDS_KB, PCG_*_SL, PCG_*_WPC, PCG_SCL_VIRT, ... */
#define PCG_DEV_OPPROF 0x10  /* PCG_OPPROF */
#define PCG_DEV_FLAGS 0x20   /* PCG_FLAGS */
#define PCG_DEV_BUILD 0x40   /* a development build of the list kernel (compile-time knobs != defaults) */

/* Build a decoding plan: classify the decoder tree exactly as the reference
 * (Fast-SSC for L == 1, SCL for L >= 2), flatten it to a device schedule and
 * upload it to `device`.  `frozen` must be strictly ascending indices < N.
 * crc_kind: PCG_CRC_NONE/8/11/16/32.  L <= 32. */
int pcg_plan_create(pcg_plan** plan,
                    uint32_t N,
                    uint32_t L,
                    const uint32_t* frozen,
                    uint32_t n_frozen,
                    int systematic,
                    int crc_kind,
                    int device);

/* An adaptive plan (makeDecoder's "mixed" = AdaptiveFloat, decoder.cpp:40-41, 75;
 * adaptive_float.cpp:33-45): pcg_decode_f32 first decodes every frame with Fast-SSC, then
 * re-decodes the frames whose detector check failed with CRC-aided SCL (list size L); a
 * re-decoded frame reports the SCL output and ok flag.  metrics: the SCL path metrics of
 * re-decoded frames, 0 for frames Fast-SSC settled.  Asynchronous (the failed-frame list
 * stays on the device).  L < 2 creates a plain Fast-SSC plan.  Fails like both decoders'
 * constructors (PCG_E_FROZEN for frozen patterns Fast-SSC rejects). */
int pcg_plan_create_adaptive(pcg_plan** plan,
                             uint32_t N,
                             uint32_t L,
                             const uint32_t* frozen,
                             uint32_t n_frozen,
                             int systematic,
                             int crc_kind,
                             int device);

/* Decode F frames.  llr: device pointer, F x N float32 (natural order, LLR > 0
 * <=> bit 0).  info: device pointer, F x ceil(K/8) bytes (MSB-first info bits,
 * exactly Decoder::getDecodedInformationBits).  ok: device pointer to F bytes
 * (Decoder::decode's return value) or NULL.  metrics: device pointer, F x L
 * floats of the final ordered SCL path metrics (unused path slots = 0), or NULL
 * (ignored for L == 1).  stream: hipStream_t or NULL for the null stream.
 * Asynchronous with respect to the host. */
int pcg_decode_f32(pcg_plan* plan,
                   const float* llr,
                   uint64_t F,
                   uint8_t* info,
                   uint8_t* ok,
                   float* metrics,
                   void* stream);

/* Same contract with HOST pointers; synchronous.  Streams the batch through
 * device buffers in chunks. */
int pcg_decode_f32_host(pcg_plan* plan,
                        const float* llr,
                        uint64_t F,
                        uint8_t* info,
                        uint8_t* ok,
                        float* metrics);

/* Fast-SSC float plans (L == 1): decode as pcg_decode_f32 and also write each frame's soft
 * codeword -- the reference's root FloatContainer word for word (Decoder::getSoftCodeword,
 * decoder.cpp:147; the leaf decoders' float outputs combined by the full 32-bit XOR of
 * RateRNode, fastssc_avx_float.cpp:148-792).  soft: device F x N floats.  Runs the
 * one-codeword-per-wave kernel (slower than pcg_decode_f32).  PCG_E_UNSUPPORTED for list,
 * 8-bit and adaptive plans and for N whose state exceeds a CU's LDS (N > 16384). */
int pcg_decode_f32_soft(pcg_plan* plan,
                        const float* llr,
                        uint64_t F,
                        uint8_t* info,
                        uint8_t* ok,
                        float* soft,
                        void* stream);

/* Same with HOST pointers; synchronous. */
int pcg_decode_f32_soft_host(pcg_plan* plan,
                             const float* llr,
                             uint64_t F,
                             uint8_t* info,
                             uint8_t* ok,
                             float* soft);

/* An 8-bit fixed-point plan: the reference's "char" decoders (FastSscFipChar for L == 1,
 * SclFipChar for L >= 2; L <= 32), classified and computed exactly as they are
 * (saturating int8 LLRs, integer path metrics).  Decode int8 frames with pcg_decode_i8, or
 * float frames with pcg_decode_f32 (quantised in the kernel as CharContainer::insertLlr
 * does, bitcontainer.cpp:449-516).  `metrics` of such plans are the integer SCL path
 * metrics as floats (exact).  Non-systematic decoding follows the reference's intent
 * (re-encode, then extract); for N < 256 the reference's own output is undefined there
 * (DESIGN.md Q9). */
int pcg_plan_create_char(pcg_plan** plan,
                         uint32_t N,
                         uint32_t L,
                         const uint32_t* frozen,
                         uint32_t n_frozen,
                         int systematic,
                         int crc_kind,
                         int device);

/* The 8-bit adaptive decoder AdaptiveChar (adaptive_char.cpp:14-45; pcsim's 8-bit list
 * decoding, simulator.cpp:722-727): FastSscFipChar for every frame, SclFipChar for the
 * frames whose check failed, as pcg_plan_create_adaptive does for the float decoders. */
int pcg_plan_create_adaptive_char(pcg_plan** plan,
                                  uint32_t N,
                                  uint32_t L,
                                  const uint32_t* frozen,
                                  uint32_t n_frozen,
                                  int systematic,
                                  int crc_kind,
                                  int device);

/* Decode F frames of int8 LLRs (device pointer, F x N bytes) with an 8-bit plan; outputs
 * as pcg_decode_f32.  PCG_E_ARG for a float plan.  Asynchronous. */
int pcg_decode_i8(pcg_plan* plan,
                  const int8_t* llr,
                  uint64_t F,
                  uint8_t* info,
                  uint8_t* ok,
                  float* metrics,
                  void* stream);

/* Same contract with HOST pointers; synchronous. */
int pcg_decode_i8_host(pcg_plan* plan,
                       const int8_t* llr,
                       uint64_t F,
                       uint8_t* info,
                       uint8_t* ok,
                       float* metrics);

int pcg_plan_describe(const pcg_plan* plan, pcg_plan_desc* desc);

/* Name of the kernel a decode on this plan launches (e.g. "sclls_kernel<8>",
 * "scs_kernel"), as it appears in rocprofv3 kernel traces; "" for NULL. */
const char* pcg_plan_kernel_name(const pcg_plan* plan);

/* Compile (hiprtc, at run time) and load a kernel specialised to this plan's code: the
 * LDS-resident Fast-SSC kernel with the plan's decoder tree as a compile-time schedule, the
 * lane-serial list kernel with the plan's layout and constants as literals, and for 8-bit
 * plans the lane-serial FastSscFipChar / SclFipChar kernels with their constants and layout as
 * literals (sccs_rtc_kernel / scl_char_rtc_kernel) -- the same device code and arithmetic as
 * the interpreter kernels, so the same outputs bit for bit.  An adaptive plan specialises both
 * of its stages.  This
 * replaces the reference's per-code decoder object tree (FastSscAvx::createDecoder,
 * fastssc_avx_float.cpp:797-896; SclAvx::createDecoder, scl_avx_float.cpp:624-651) with
 * per-code machine code.  Code objects are cached per process, in the library's shipped
 * cache (<dir of libpcg.so>/rtc, filled at build time for the catalogue of
 * antpolarcodes_amd/rtc_codes.py: the benchmark configurations and a validation catalogue) and
 * on disk (PCG_RTC_CACHE); a code in none of them takes tens of seconds of hiprtc once.
 * Plans do this by themselves: with a cached code object from their first decode, otherwise
 * in a background thread from their first decode of >= 8192 frames, switching once it is
 * ready (PCG_RTC=0 never, PCG_RTC=1 at the first decode, waiting).  PCG_E_UNSUPPORTED for
 * the 8-bit Fast-SSC plans that run the one-codeword-per-wave kernel and with PCG_OPPROF; on
 * a host-only plan it only compiles.  On failure (no hiprtc, a device of another
 * architecture) the plan keeps decoding with the interpreter kernel.  Plans of one code
 * share one compile; pcg_plan_destroy never waits for it, process exit does (with a notice
 * on stderr; PCG_RTC_EXIT_WAIT=<s> bounds that wait).  The first compile a process starts is
 * preceded by a short warm-up compile (~1-2 s, loading hiprtc's compiler) on the calling
 * thread, so the first pcg_plan_specialize_async -- or the first decode of >= 8192 frames
 * that starts a compile -- can block for that long. */
int pcg_plan_specialize(pcg_plan* plan);

/* Start pcg_plan_specialize without waiting: the plan switches at a later decode (or
 * pcg_plan_specialize) once the code object is ready.  Returns without waiting for the
 * compile (only the process's first compile is preceded by the warm-up above). */
int pcg_plan_specialize_async(pcg_plan* plan);

/* SCL plans: the metric path 0 starts every frame of later decode calls with.  0 (the
 * default) is a freshly constructed reference decoder; passing the previous frame's final
 * metrics[0] reproduces a reference decoder instance reused frame after frame (its
 * PathList never resets mMetric, scl_avx_float.cpp:31, 99-109).  For the
 * 8-bit plans the value is converted to the integer metric.  Ignored by Fast-SSC. */
int pcg_plan_set_initial_metric(pcg_plan* plan, float metric0);

void pcg_plan_destroy(pcg_plan* plan);

const char* pcg_last_error(void);

/* Number of HIP devices visible (0 without a GPU); never fails. */
int pcg_device_count(void);

/* ---- rate matching: Puncturer --------------------------------------------------------
 * Puncturer(blockLength = E, frozenBitPositions): parent length N = next power of two
 * >= E; the first N - E entries of `frozen` (as given; frozen_bits returns them
 * ascending) are punctured; PCG_E_ARG with the reference's std::out_of_range text
 * ("Number of required puncturing positions exceeds frozen bit positions!") when the
 * frozen set is too small.  device < 0: host-only (positions, no device tables). */
typedef struct pcg_puncturer pcg_puncturer;

int pcg_puncturer_create(pcg_puncturer** punc,
                         uint32_t E,
                         const uint32_t* frozen,
                         uint32_t n_frozen,
                         int device);

/* E, N and (if `positions` is not NULL) the E kept parent positions, ascending
 * (Puncturer::blockLength / parentBlockLength / blockOutputPositions). */
int pcg_puncturer_describe(const pcg_puncturer* punc, uint32_t* E, uint32_t* N, uint32_t* positions);

/* Device buffers, asynchronous on `stream`:
 *   depuncture  in F x E floats -> out F x N floats, punctured positions = +0.0f
 *   puncture    in F x N floats -> out F x E floats
 *   puncture_packed  in F x N/8 MSB-first bytes -> out F x E/8 (E, N multiples of 8) */
int pcg_depuncture_f32(const pcg_puncturer* punc, const float* in, uint64_t F, float* out, void* stream);
int pcg_puncture_f32(const pcg_puncturer* punc, const float* in, uint64_t F, float* out, void* stream);
int pcg_puncture_packed(const pcg_puncturer* punc, const uint8_t* in, uint64_t F, uint8_t* out, void* stream);

void pcg_puncturer_destroy(pcg_puncturer* punc);

/* Decode F punctured frames: llr is F x E (device), depunctured on the device and decoded
 * with `plan` (whose N must equal the puncturer's parent length).  Outputs as
 * pcg_decode_f32.  Float list plans depuncture inside the decode kernel (each wave its
 * codeword group, into its scratch: one launch, no staging buffer); the other plans
 * depuncture into a plan staging buffer first (reused across calls, ordered after the
 * plan's previous decode).  Stream-ordered. */
int pcg_decode_punctured_f32(pcg_plan* plan,
                             const pcg_puncturer* punc,
                             const float* llr,
                             uint64_t F,
                             uint8_t* info,
                             uint8_t* ok,
                             float* metrics,
                             void* stream);

/* ---- frame source: encoder, random information, BPSK-AWGN channel ---------------------- */
typedef struct pcg_encoder pcg_encoder;

/* ButterflyFipPacked(N, frozen) + setSystematic + setErrorDetection(crc_kind). */
int pcg_encoder_create(pcg_encoder** enc,
                       uint32_t N,
                       const uint32_t* frozen,
                       uint32_t n_frozen,
                       int systematic,
                       int crc_kind,
                       int device);

/* info: device F x ceil(K/8) bytes; the detector's check bits are written into it in
 * place (as encode_vector does to its caller's buffer).  code: device F x N/8 bytes,
 * MSB-first (Encoder::getEncodedData). */
int pcg_encode(pcg_encoder* enc, uint8_t* info, uint64_t F, uint8_t* code, void* stream);

void pcg_encoder_destroy(pcg_encoder* enc);

/* Uniform random information bytes (device F x ceil(K/8)), bits past K cleared:
 * Philox4x32-10 keyed by `seed`, counter = (frame, byte block). */
int pcg_random_info(uint8_t* info, uint64_t F, uint32_t K, uint64_t seed, void* stream);

/* BPSK (bit 0 -> +1) + AWGN of standard deviation sigma + LLR = 2 y / sigma^2 over n
 * packed code bits per frame (device code F x n/8 -> llr F x n floats, n % 8 == 0).
 * sigma <= 0: noiseless, llr = +-1.  Noise from Philox4x32-10 keyed by `seed`. */
int pcg_bpsk_awgn_f32(const uint8_t* code, uint64_t F, uint32_t n, float sigma, uint64_t seed, float* llr,
                      void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PCG_H */
