/* -*- c++ -*- */
// PolarCode::Decoding -- drop-in for the reference's decoder interface
// (include/polarcode/decoding/decoder.h:40-211 of david13pod/antPolarCodes).
//
// The virtual base keeps the reference's members, names, argument meanings and error
// behaviour (BitContainer input/output containers, unsigned char* packed output,
// mExternalContainers), so reference-style subclasses compile unchanged.  The
// implementations (GpuFastSscFloat, GpuSclFloat, ... -- also reachable under the
// reference's class names through <polarcode/decoding/fastssc_avx_float.h> etc.) run the
// MI355X kernels through the C ABI of include/pcg.h.  New: decodeBatch() for F frames per
// call (host buffers), decodeBatchDevice() (device buffers, asynchronous on a HIP stream)
// and decodeBatchI8().
#ifndef PCA_DECODER_H
#define PCA_DECODER_H

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include <polarcode/bitcontainer.h>
#include <polarcode/errordetection/errordetector.h>

struct pcg_plan;

namespace PolarCode {
namespace Decoding {

enum DecoderType { tFlexible, tFixed, tDepthFirst, tScan, tFastSscan };

class Decoder
{
private:
    size_t mDecoderDuration;

protected:
    ErrorDetection::Detector* mErrorDetector; ///< Error detecting object (not owned)
    size_t mBlockLength;                      ///< Length of the Polar Code
    bool mSystematic;                         ///< Whether to use systematic coding
    BitContainer* mLlrContainer;              ///< Soft-input container
    BitContainer* mBitContainer;              ///< (optionally soft-) Output bit container
    unsigned char* mOutputContainer;          ///< Decoded information bytes, (K+7)/8
    std::vector<unsigned> mFrozenBits;        ///< Indices for frozen bits
    bool mExternalContainers;                 ///< On destruction, do not delete containers

public:
    Decoder();
    virtual ~Decoder();

    /// Decode the signal given by setSignal(); returns the detector's verdict.
    virtual bool decode() = 0;
    /// setSignal + decode + getDecodedInformationBits (decoder.cpp:154-167).
    bool decode_vector(const float* pLlr, void* pData);
    /// setSignal(const char*) + decode + getDecodedInformationBits (decoder.cpp:169-181).
    bool decode_vector(const char* pLlr, void* pData);
    /// Nanoseconds of the last decode_vector call.
    size_t duration_ns() { return mDecoderDuration; }

    virtual void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits);
    std::vector<unsigned> frozenBits() { return mFrozenBits; }
    size_t blockLength();
    size_t infoLength();

    BitContainer* inputContainer();  ///< mLlrContainer
    BitContainer* outputContainer(); ///< mBitContainer
    unsigned char* packedOutput();   ///< mOutputContainer

    virtual void setSystematic(bool sys);
    bool isSystematic();
    virtual void setErrorDetection(ErrorDetection::Detector* pDetector);
    std::string getErrorDetectionMode()
    {
        return std::string(mErrorDetector->getType() + "-" + std::to_string(mErrorDetector->getCheckBitCount()));
    }
    virtual size_t getListSize() { return 1; }
    /// mLlrContainer->insertLlr(pLlr) (decoder.cpp:138).
    virtual void setSignal(const float* pLlr);
    /// mLlrContainer->insertLlr(pLlr) (decoder.cpp:140): float containers convert the
    /// bytes, char containers copy them.
    void setSignal(const char* pLlr);
    void getDecodedInformationBits(void* pData);
    /// mBitContainer->getSoftBits (decoder.cpp:147).
    void getSoftCodeword(void* pData);
    /// mBitContainer->getSoftInformation (decoder.cpp:149-152).
    void getSoftInformation(void* pData);

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

class UndefinedDecoder : public Decoder
{
public:
    UndefinedDecoder();
    ~UndefinedDecoder();
    bool decode() override;
};

/// Output container of the GPU float decoders (outputContainer()): after a Fast-SSC float
/// decode (N <= 16384) it holds the soft codeword word for word (FloatContainer::getSoftBits
/// of the reference); otherwise the decoded codeword's hard decisions as sign bits
/// (+0.0 / -0.0) -- getPackedBits / getFloatBits / getPackedInformationBits exact -- which
/// the soft accessors return: the selected path's signed hard decisions, whose signs are the
/// reference's (only the signs of its list decoders' bit floats are observable).
class DecodedFloatContainer : public FloatContainer
{
    bool mSoft = false;

public:
    DecodedFloatContainer(size_t size, const std::vector<unsigned>& frozenBits) : FloatContainer(size, frozenBits) {}
    void setSoft(bool soft) { mSoft = soft; }
    bool isSoft() const { return mSoft; }
    void getSoftBits(void* pData) override;
    void getSoftInformation(void* pData) override;
};

/// Output container of the GPU 8-bit decoders: hard decisions as char bits (0 -> 127,
/// 1 -> -128, CharContainer::insertPackedBits), which the soft accessors return.
class DecodedCharContainer : public CharContainer
{
public:
    DecodedCharContainer(size_t size, const std::vector<unsigned>& frozenBits) : CharContainer(size, frozenBits) {}
    void getSoftBits(void* pData) override;
    void getSoftInformation(void* pData) override;
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
    /// the detector / systematic flag the plan evaluates: mErrorDetector / mSystematic,
    /// except for the adaptive decoders, which (as AdaptiveFloat, adaptive_float.cpp:47-57)
    /// pass them to their stages and leave their own members untouched
    ErrorDetection::Detector* mStageDetector;
    bool mStageSystematic = true;
    /// SCL: path 0's final metric of the last decode(), the next decode()'s start metric --
    /// one reference decoder instance reused frame after frame
    float mCarry = 0.0f;
    void ensurePlan();
    void releasePlan();
    void setupContainers();
    void fillHardCodeword();

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

/// CRC-aided SCL (SclAvxFloat, scl_avx_float.cpp) on the GPU; listSize 2..32 (any value).
class GpuSclFloat : public GpuDecoder
{
public:
    GpuSclFloat(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int device = 0)
        : GpuDecoder(blockLength, listSize, frozenBits, device)
    {
    }
};

/// AdaptiveFloat (adaptive_float.cpp:14-57): Fast-SSC, then CRC-aided SCL for the frames
/// whose check fails -- per frame, on the GPU, in one batched call.
class GpuAdaptiveFloat : public GpuDecoder
{
public:
    GpuAdaptiveFloat(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int device = 0);
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

/// AdaptiveMixed (adaptive_mixed.cpp:14-78; pcsim's default precision 832): FastSscFipChar
/// over the (quantised) float frames, then the float SCL for the frames whose check fails.
/// Composed of two GPU decoders like the reference composes two CPU ones.
class GpuAdaptiveMixed : public Decoder
{
    GpuFastSscChar* mFastDecoder;
    GpuSclFloat* mListDecoder;
    size_t mListSize;

public:
    GpuAdaptiveMixed(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                     int device = 0);
    ~GpuAdaptiveMixed() override;
    bool decode() override;
    void setSystematic(bool sys) override;
    void setErrorDetection(ErrorDetection::Detector* pDetector) override;
    void setSignal(const float* pLlr) override;
    size_t getListSize() override { return mListSize; }
    /// Fast stage over all frames, list stage over the failures (host buffers).
    bool decodeBatch(const float* llr, size_t F, uint8_t* info, uint8_t* ok = nullptr,
                     float* metrics = nullptr) override;
};

/// makeDecoder (decoder.cpp:54-87): decoder_impl 1 = float (Fast-SSC for listSize 1, else
/// SCL), 2 = AdaptiveFloat (listSize >= 2), 3 = SCAN (not part of this build:
/// std::logic_error), every other value = the 8-bit decoders (FastSscFipChar / SclFipChar),
/// the default 0 included.  Always installs a CRC-8 detector (the reference's Q5 behaviour).
Decoder* makeDecoder(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                     int decoder_impl = 0);

/// create (decoder.cpp:26-52).  "char" -> 8-bit, "float" (and this build's "gpu") -> the
/// MI355X float decoders, "mixed" -> AdaptiveFloat; listSize < 2 turns every non-char type
/// into Fast-SSC float; "scan" is outside this build (std::logic_error); unknown strings
/// raise std::logic_error("Unknown PolarDecoder type!") exactly as the reference.
Decoder* create(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                std::string decoderType);

} // namespace Decoding
} // namespace PolarCode

#endif
