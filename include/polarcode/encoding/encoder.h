/* -*- c++ -*- */
// PolarCode::Encoding::Encoder -- the reference's encoder skeleton-class
// (include/polarcode/encoding/encoder.h:24-151, src/polarcode/encoding/encoder.cpp of
// david13pod/antPolarCodes), unchanged in members and semantics: encode() is the pure
// virtual algorithm, encode_vector() = setInformation + encode + getEncodedData, the
// bits live in a BitContainer (include/polarcode/bitcontainer.h).  ButterflyFipPacked
// is in <polarcode/encoding/butterfly_fip_packed.h>; the batched device encoder is
// pcg_encode (include/pcg.h).
#ifndef PCA_ENCODER_H
#define PCA_ENCODER_H

#include <cstddef>
#include <string>
#include <vector>

#include <polarcode/bitcontainer.h>
#include <polarcode/errordetection/errordetector.h>

namespace PolarCode {
namespace Encoding {

class Encoder
{
private:
    size_t mEncoderDuration;

protected:
    ErrorDetection::Detector* mErrorDetector; ///< Error detecting object (not owned)
    size_t mBlockLength;                      ///< Block length of the Polar Code
    bool mSystematic;                         ///< Whether to use systematic coding
    bool mCodewordReady;                      ///< mBitContainer already holds the bits to encode
    unsigned char* xmInputData;               ///< Bits to encode (setInformation / setCodeword)
    BitContainer* mBitContainer;              ///< Internal bit memory (owned)
    std::vector<unsigned> mFrozenBits;        ///< Indices for frozen bits

public:
    Encoder();
    virtual ~Encoder();
    virtual void encode() = 0; ///< Execute the encoding algorithm.

    /// setInformation(pInfo) + encode() + getEncodedData(pCode) (encoder.cpp:79-90).
    void encode_vector(void* pInfo, void* pCode);

    /// Nanoseconds of the last encoder call (never set by the reference's encode_vector).
    size_t duration_ns() { return mEncoderDuration; }

    virtual void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits) = 0;

    size_t infoLength() { return blockLength() - mFrozenBits.size(); }
    size_t blockLength();
    std::vector<unsigned> frozenBits() { return mFrozenBits; }

    void setErrorDetection(ErrorDetection::Detector* pDetector);
    std::string getErrorDetectionMode()
    {
        return std::string(mErrorDetector->getType() + "-" + std::to_string(mErrorDetector->getCheckBitCount()));
    }

    void setSystematic(bool sys);
    bool isSystematic();

    /// Keep a pointer to the packed information bytes for the next encode() (not copied;
    /// encode() writes the detector's check bits into them, as the reference does).
    void setInformation(void* pData);
    /// Packed information bits of the container (after encode(): of the codeword).
    void getInformation(void* pData);
    /// Packed codeword bits into the container; the next encode() transforms them as given.
    void setCodeword(void* pData);
    /// Char bits (MSB of each byte) into the container.
    void setCharCodeword(void* cData);
    /// Float bits (sign bits) into the container.
    void setFloatCodeword(void* fData);
    /// Packed code bits (N/8 bytes) of the last encode().
    void getEncodedData(void* pData);
    /// Set all frozen bits to 0.
    void clearFrozenBits();
};

class UndefinedEncoder : public Encoder
{
public:
    UndefinedEncoder();
    ~UndefinedEncoder();
    void initialize(size_t, const std::vector<unsigned>&) override;
    void encode() override;
};

} // namespace Encoding
} // namespace PolarCode

#endif
