/* -*- c++ -*- */
// PolarCode::Decoding -- drop-in for the reference's decoder interface
// (include/polarcode/decoding/decoder.h:40-211 of david13pod/antPolarCodes).
//
// The virtual base keeps the reference's names, argument meanings and error
// behaviour; the implementations (GpuFastSscFloat, GpuSclFloat) run the
// MI355X kernels through the C ABI of include/pcg.h.  New: decodeBatch() for F
// frames per call (host buffers) and decodeBatchDevice() (device buffers,
// asynchronous on a HIP stream).
#ifndef PCA_DECODER_H
#define PCA_DECODER_H

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include <polarcode/errordetection/errordetector.h>

struct pcg_plan;

namespace PolarCode {
namespace Decoding {

class Decoder
{
protected:
    size_t mDecoderDuration = 0;
    ErrorDetection::Detector* mErrorDetector; ///< not owned (as in the reference)
    size_t mBlockLength = 0;
    bool mSystematic = true;
    std::vector<unsigned> mFrozenBits;
    std::vector<float> mLlr;                  ///< setSignal() input (one frame)
    std::vector<int8_t> mLlr8;                ///< setSignal(const char*) input of 8-bit decoders
    bool mSignalI8 = false;                   ///< the pending frame is mLlr8
    std::vector<unsigned char> mOutputContainer;
    bool mLastOk = false;
    bool mCharContainer = false;              ///< 8-bit decoder: setSignal(const char*) keeps the bytes
    std::vector<float> mSoftCodeword;         ///< soft codeword of the last decode() (empty: none)

public:
    Decoder();
    virtual ~Decoder();

    /// Decode the frame given by setSignal(); returns the detector's verdict.
    virtual bool decode() = 0;
    /// setSignal + decode + getDecodedInformationBits (decoder.cpp:154-167).
    bool decode_vector(const float* pLlr, void* pData);
    /// setSignal(const char*) + decode + getDecodedInformationBits (decoder.cpp:169-181).
    bool decode_vector(const char* pLlr, void* pData);
    size_t duration_ns() { return mDecoderDuration; }

    virtual void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits);
    std::vector<unsigned> frozenBits() { return mFrozenBits; }
    size_t blockLength() { return mBlockLength; }
    size_t infoLength() { return mBlockLength - mFrozenBits.size(); }
    unsigned char* packedOutput() { return mOutputContainer.data(); }

    virtual void setSystematic(bool sys);
    bool isSystematic() { return mSystematic; }
    virtual void setErrorDetection(ErrorDetection::Detector* pDetector);
    std::string getErrorDetectionMode()
    {
        return mErrorDetector->getType() + "-" + std::to_string(mErrorDetector->getCheckBitCount());
    }
    virtual size_t getListSize() { return 1; }
    virtual void setSignal(const float* pLlr);
    /// 8-bit LLRs (non-virtual, as in the reference, decoder.h:170): float decoders convert
    /// them (FloatContainer::insertLlr(const char*), bitcontainer.cpp:202-207); 8-bit
    /// decoders take them as they are (CharContainer::insertLlr).
    void setSignal(const char* pLlr);
    void getDecodedInformationBits(void* pData);
    /// The last decode()'s soft codeword, N floats (FloatContainer::getSoftBits,
    /// bitcontainer.cpp:294-297): the root bit container word for word.  Available from
    /// the Fast-SSC float decoder; std::logic_error for decoders whose GPU kernels keep
    /// hard decisions only (SCL, 8-bit, adaptive).
    void getSoftCodeword(void* pData);
    /// The soft codeword at the information positions, K floats
    /// (FloatContainer::getSoftInformation, bitcontainer.cpp:331-339).
    void getSoftInformation(void* pData);
    /// Direct access to the decoder's input LLRs (N floats) and soft output (N floats,
    /// empty before a soft-capable decode).  The reference returns its BitContainer
    /// objects here (decoder.h:107-108); this build has no container classes.
    float* inputContainer() { return mLlr.data(); }
    float* outputContainer() { return mSoftCodeword.empty() ? nullptr : mSoftCodeword.data(); }

    /// Batched decode of F frames (host memory): llr F x N, info F x ceil(K/8),
    /// ok F (nullable), metrics F x L (nullable, list decoders only).  Returns true if
    /// every frame passed the detector.  The default decodes frame by frame through
    /// decode_vector (metrics left untouched); the GPU decoders run one batched launch.
    virtual bool decodeBatch(const float* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                             float* metrics = nullptr);
    /// Same with device pointers, asynchronous on `hipStream` (null = default stream).
    /// The default raises std::logic_error (a CPU decoder has no device path).
    virtual void decodeBatchDevice(const float* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                                   float* metrics = nullptr, void* hipStream = nullptr);
    /// Batched decode of F frames of int8 LLRs (host memory); default: decode_vector(const char*).
    virtual bool decodeBatchI8(const int8_t* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                               float* metrics = nullptr);
};

/// Shared GPU plumbing: owns one pcg_plan, rebuilt when code / detector / systematic
/// flag change.
class GpuDecoder : public Decoder
{
protected:
    size_t mListSize;
    int mDevice;
    pcg_plan* mPlan = nullptr;
    int mPlanKind = -2;
    bool mPlanSys = true;
    bool mAdaptive = false; ///< pcg_plan_create_adaptive (Fast-SSC first, SCL for failures)
    bool mFixed = false;    ///< pcg_plan_create_char (the reference's 8-bit decoders)
    /// SCL: path 0's final metric of the last decode(), the next decode()'s start metric --
    /// one reference decoder instance reused frame after frame
    float mCarry = 0.0f;
    void ensurePlan();
    void releasePlan();

public:
    GpuDecoder(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int device);
    ~GpuDecoder() override;
    bool decode() override;
    void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits) override;
    void setSystematic(bool sys) override;
    void setErrorDetection(ErrorDetection::Detector* pDetector) override;
    size_t getListSize() override { return mListSize; }
    bool decodeBatch(const float* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                     float* metrics = nullptr) override;
    void decodeBatchDevice(const float* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                           float* metrics = nullptr, void* hipStream = nullptr) override;
    bool decodeBatchI8(const int8_t* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                       float* metrics = nullptr) override;
    /// int8 frames in device memory (8-bit decoders only), asynchronous on `hipStream`.
    void decodeBatchDeviceI8(const int8_t* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                             float* metrics = nullptr, void* hipStream = nullptr);
    bool isFixedPoint() const { return mFixed; }
    /// SCL: the start metric the next decode() carries (0 after construction).
    float carriedMetric() const { return mCarry; }
    int device() const { return mDevice; }
};

/// Fast-SSC (FastSscAvxFloat, fastssc_avx_float.cpp) on the GPU.
class GpuFastSscFloat : public GpuDecoder
{
public:
    GpuFastSscFloat(size_t blockLength, const std::vector<unsigned>& frozenBits, int device = 0)
        : GpuDecoder(blockLength, 1, frozenBits, device)
    {
    }
};

/// CRC-aided SCL (SclAvxFloat, scl_avx_float.cpp) on the GPU; listSize 2..32.
class GpuSclFloat : public GpuDecoder
{
public:
    GpuSclFloat(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                int device = 0)
        : GpuDecoder(blockLength, listSize, frozenBits, device)
    {
    }
};

/// makeDecoder (decoder.cpp:54-87): L == 1 -> Fast-SSC, else SCL; always installs
/// a CRC-8 detector (the reference's Q5 behaviour).
/// AdaptiveFloat (adaptive_float.cpp:14-45): Fast-SSC, then CRC-aided SCL for the frames
/// whose check fails -- per frame, on the GPU, in one batched call.
class GpuAdaptiveFloat : public GpuDecoder
{
public:
    GpuAdaptiveFloat(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                     int device = 0);
};

/// FastSscFipChar (fastssc_fip_char.cpp) on the GPU: 8-bit saturating LLRs.
class GpuFastSscChar : public GpuDecoder
{
public:
    GpuFastSscChar(size_t blockLength, const std::vector<unsigned>& frozenBits, int device = 0);
};

/// SclFipChar (scl_fip_char.cpp) on the GPU: 8-bit LLRs, integer path metrics; listSize 2..32.
class GpuSclChar : public GpuDecoder
{
public:
    GpuSclChar(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int device = 0);
};

/// AdaptiveChar (adaptive_char.cpp:14-45; pcsim's 8-bit list decoding): FastSscFipChar, then
/// SclFipChar for the frames whose check fails.  Not reachable through create(), as in the reference.
class GpuAdaptiveChar : public GpuDecoder
{
public:
    GpuAdaptiveChar(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                    int device = 0);
};

/// decoder_impl as in decoder.cpp:54-87: 0 = char (FastSscFipChar / SclFipChar), 1 = float
/// (Fast-SSC / SCL), 2 = AdaptiveFloat (list size >= 2); SCAN (3) is not part of this build.
Decoder* makeDecoder(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                     int decoder_impl = 1);

/// create (decoder.cpp:26-52).  "gpu" and "float" select the MI355X float decoders
/// (listSize < 2 -> Fast-SSC), "char" the 8-bit ones, "mixed" AdaptiveFloat; "scan" is a
/// reference decoder outside this build and raises std::logic_error; unknown strings raise
/// std::logic_error("Unknown PolarDecoder type!") exactly as the reference.
Decoder* create(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                std::string decoderType);

} // namespace Decoding
} // namespace PolarCode

#endif
