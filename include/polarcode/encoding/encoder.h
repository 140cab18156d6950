/* -*- c++ -*- */
// PolarCode::Encoding::Encoder (encoder.h:24-151 of the reference) and the packed
// butterfly encoder (butterfly_fip_packed.cpp:45-70), host-side.  Used to build
// frames and by callers that pair it with the GPU decoders.
#ifndef PCA_ENCODER_H
#define PCA_ENCODER_H

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include <polarcode/errordetection/errordetector.h>

namespace PolarCode {
namespace Encoding {

class Encoder
{
protected:
    ErrorDetection::Detector* mErrorDetector;
    size_t mBlockLength;
    bool mSystematic;
    std::vector<unsigned> mFrozenBits;

public:
    Encoder();
    virtual ~Encoder() {}
    virtual void encode_vector(void* pInfo, void* pCode) = 0;
    virtual void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits) = 0;
    size_t blockLength() { return mBlockLength; }
    size_t infoLength() { return mBlockLength - mFrozenBits.size(); }
    std::vector<unsigned> frozenBits() { return mFrozenBits; }
    void setErrorDetection(ErrorDetection::Detector* pDetector) { mErrorDetector = pDetector; }
    std::string getErrorDetectionMode()
    {
        return mErrorDetector->getType() + "-" + std::to_string(mErrorDetector->getCheckBitCount());
    }
    void setSystematic(bool sys) { mSystematic = sys; }
    bool isSystematic() { return mSystematic; }
};

/// ButterflyFipPacked: info bytes (MSB-first, CRC generated over them first) ->
/// packed codeword bytes; systematic = transform, clear frozen, transform.
class ButterflyFipPacked : public Encoder
{
    std::vector<uint8_t> mIsFrozen;

public:
    ButterflyFipPacked(size_t blockLength, const std::vector<unsigned>& frozenBits);
    void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits) override;
    void encode_vector(void* pInfo, void* pCode) override;
};

} // namespace Encoding
} // namespace PolarCode

#endif
