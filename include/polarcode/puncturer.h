/* -*- c++ -*- */
// PolarCode::Puncturer -- rate matching by puncturing, the reference's interface
// (include/polarcode/puncturer.h:33-99, src/polarcode/puncturer.cpp:23-89 in
// david13pod/antPolarCodes), host side.  The batched device depuncturer behind it is
// pcg_depuncture_f32 / pcg_decode_punctured_f32 (include/pcg.h).
#ifndef PCA_PUNCTURER_H
#define PCA_PUNCTURER_H

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace PolarCode {

/// Next power of two >= value (32-bit bit trick, puncturer.cpp:23-33).
size_t round_up_power_of_two(size_t value);

/// [0, blockLength) minus `positions`, by the std::set_difference merge
/// (puncturer.cpp:35-49; `positions` is expected ascending, as frozen_bits returns).
std::vector<unsigned> inverse_set_difference(size_t blockLength, std::vector<unsigned> positions);

class Puncturer
{
protected:
    size_t mBlockLength;                    // punctured length E
    size_t mParentBlockLength;              // N = next power of two >= E
    std::vector<unsigned> mOutputPositions; // parent positions kept, ascending

public:
    /// The first N-E entries of frozenBitPositions are punctured; more than the frozen set
    /// holds throws std::out_of_range (puncturer.cpp:51-66).
    Puncturer(const size_t blockLength, const std::vector<unsigned> frozenBitPositions);
    virtual ~Puncturer();

    size_t blockLength() { return mBlockLength; }
    size_t parentBlockLength() { return mParentBlockLength; }
    std::vector<unsigned> blockOutputPositions() { return mOutputPositions; }

    /// pOutput[k] = pInput[outputPositions[k]], k < E.
    template <typename T>
    void puncture(T* pOutput, const T* pInput)
    {
        for (size_t k = 0; k < mOutputPositions.size(); ++k)
            pOutput[k] = pInput[mOutputPositions[k]];
    }

    /// Packed-bit variant (MSB-first bytes; E and N multiples of 8), puncturer.cpp:71-89.
    void puncturePacked(unsigned char* pOutput, const unsigned char* pInput);

    /// pOutput[0..N) = 0 (+0.0 for floats), then pOutput[outputPositions[k]] = pInput[k].
    template <typename T>
    void depuncture(T* pOutput, const T* pInput)
    {
        std::fill(pOutput, pOutput + mParentBlockLength, T(0));
        for (size_t k = 0; k < mOutputPositions.size(); ++k)
            pOutput[mOutputPositions[k]] = pInput[k];
    }
};

} // namespace PolarCode

#endif
