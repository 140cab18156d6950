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
 *   pcg_plan_destroy  <- Decoder::~Decoder decoder.cpp:104-114
 *   pcg_last_error    <- the std::exception text the reference throws
 *
 * Error model: every function returns 0 on success or a negative PCG_E* code;
 * nothing throws across the ABI.  pcg_last_error() (thread-local) describes the
 * most recent failure on the calling thread.
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
} pcg_plan_desc;

/* Build a decoding plan: classify the decoder tree exactly as the reference
 * (Fast-SSC for L == 1, SCL for L >= 2), flatten it to a device schedule and
 * upload it to `device`.  `frozen` must be strictly ascending indices < N.
 * crc_kind: PCG_CRC_NONE/8/16/32.  L <= 32. */
int pcg_plan_create(pcg_plan** plan,
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

int pcg_plan_describe(const pcg_plan* plan, pcg_plan_desc* desc);

void pcg_plan_destroy(pcg_plan* plan);

const char* pcg_last_error(void);

/* Number of HIP devices visible (0 without a GPU); never fails. */
int pcg_device_count(void);

#ifdef __cplusplus
}
#endif

#endif /* PCG_H */
