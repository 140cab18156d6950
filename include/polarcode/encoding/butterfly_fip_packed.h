/* -*- c++ -*- */
// ButterflyFipPacked -- the reference's packed butterfly encoder
// (include/polarcode/encoding/butterfly_fip_packed.h, src/polarcode/encoding/
// butterfly_fip_packed.cpp:19-70): Detector::generate over the information bytes, bits
// into a PackedContainer, the polar transform x[i] ^= x[i + 2^s] over all stages;
// systematic = transform, clear frozen bits, transform.  Host side, one frame; F frames on
// the device: pcg_encode (include/pcg.h).
#ifndef PCA_BUTTERFLY_FIP_PACKED_H
#define PCA_BUTTERFLY_FIP_PACKED_H

#include <polarcode/encoding/encoder.h>

namespace PolarCode {
namespace Encoding {

class ButterflyFipPacked : public Encoder
{
    void transform();

public:
    ButterflyFipPacked();
    ButterflyFipPacked(size_t blockLength);
    ButterflyFipPacked(size_t blockLength, const std::vector<unsigned>& frozenBits);
    ~ButterflyFipPacked();

    void encode() override;
    void initialize(size_t blockLength, const std::vector<unsigned>& frozenBits) override;
};

} // namespace Encoding
} // namespace PolarCode

#endif
