/* -*- c++ -*- */
// PolarCode::BitContainer family -- the reference's bit-format containers
// (include/polarcode/bitcontainer.h:23-291, src/polarcode/bitcontainer.cpp of
// david13pod/antPolarCodes), host-side and scalar.  Same classes, members and
// semantics: float "bits" are sign bits (0 -> +0.0, 1 -> -0.0), char bits are
// 127 / -128, packed bits are MSB-first bytes.  The GPU decoders keep their
// state on the device; these containers are their host-side input/output
// objects (Decoder::inputContainer / outputContainer) and the encoder's
// internal memory, exactly as in the reference.
#ifndef PCA_BITCONTAINER_H
#define PCA_BITCONTAINER_H

#include <cstddef>
#include <vector>

namespace PolarCode {

/// The BitContainer skeleton-class (bitcontainer.h:23-155).
class BitContainer
{
    void clear();
    void calculateLUT();

protected:
    size_t mElementCount;              ///< The fixed number of bits stored in this container.
    std::vector<unsigned> mFrozenBits; ///< The set of frozen bits.
    unsigned mInformationBitCount;     ///< Parameter K.
    unsigned* mLUT;                    ///< Information positions, ascending (bitcontainer.cpp:68-84).

public:
    BitContainer();
    BitContainer(size_t size);
    BitContainer(size_t size, const std::vector<unsigned>& frozenBits);
    virtual ~BitContainer();

    virtual void setSize(size_t newSize) = 0;
    size_t size();
    void setFrozenBits(const std::vector<unsigned>& frozenBits);

    virtual void insertPackedBits(const void* pData) = 0;
    virtual void insertPackedInformationBits(const void* pData) = 0;
    virtual void insertCharBits(const void* pData) = 0;
    virtual void insertLlr(const float* pLlr) = 0;
    virtual void insertLlr(const char* pLlr) = 0;
    virtual void getPackedBits(void* pData) = 0;
    virtual void getPackedInformationBits(void* pData) = 0;
    virtual void getSoftBits(void* pData) = 0;
    virtual void getFloatBits(float* pData) = 0;
    virtual void getSoftInformation(void* pData) = 0;
    virtual void resetFrozenBits() = 0;
};

/// Bits in single-precision sign-bit format (bitcontainer.h:169-200).
class FloatContainer : public BitContainer
{
    float* mData;
    bool mDataIsExternal;

public:
    FloatContainer();
    FloatContainer(size_t size);
    FloatContainer(float* external, size_t size);
    FloatContainer(size_t size, const std::vector<unsigned>& frozenBits);
    ~FloatContainer();
    void setSize(size_t newSize) override;
    void insertPackedBits(const void* pData) override;
    void insertPackedInformationBits(const void* pData) override;
    void insertCharBits(const void* pData) override;
    void insertLlr(const float* pLlr) override;
    void insertLlr(const char* pLlr) override;
    void getPackedBits(void* pData) override;
    void getPackedInformationBits(void* pData) override;
    void getSoftBits(void* pData) override;
    void getFloatBits(float* pData) override;
    void getSoftInformation(void* pData) override;
    void resetFrozenBits() override;

    float* data();
};

/// Bits / LLRs as eight-bit integers (bitcontainer.h:211-239).  insertLlr(const float*)
/// quantises exactly as the reference: N >= 32 cvtps_epi32 (round to nearest even, NaN and
/// |x| >= 2^31 -> INT_MIN) then saturating packs; 8 <= N < 32 clamp to [-128, 127] with
/// MAXPS/MINPS semantics, then round to nearest even; N < 8 fmin/fmax clamp, round()
/// (half away from zero) (bitcontainer.cpp:27-39, 449-516).
class CharContainer : public BitContainer
{
    char* mData;
    bool mDataIsExternal;

public:
    CharContainer();
    CharContainer(size_t size);
    CharContainer(char* external, size_t size);
    CharContainer(size_t size, const std::vector<unsigned>& frozenBits);
    ~CharContainer();
    void setSize(size_t newSize) override;
    void insertPackedBits(const void* pData) override;
    void insertPackedInformationBits(const void* pData) override;
    void insertCharBits(const void* pData) override;
    void insertLlr(const float* pLlr) override;
    void insertLlr(const char* pLlr) override;
    void getPackedBits(void* pData) override;
    void getPackedInformationBits(void* pData) override;
    void getSoftBits(void* pData) override;
    void getFloatBits(float* pData) override;
    void getSoftInformation(void* pData) override;
    void resetFrozenBits() override;

    char* data();
};

/// Packed MSB-first bits for encoding (bitcontainer.h:248-291).  As in the reference, a
/// code shorter than 256 bits sits at the END of a 256-bit buffer (mFakeSize), and
/// insertCharBits() writes at the buffer's start regardless (the reference's behaviour,
/// DESIGN.md Q9).
class PackedContainer : public BitContainer
{
    char* mData;
    unsigned long* mInformationMask;
    size_t mFakeSize;
    bool mDataIsExternal;

    void buildInformationMask();
    size_t offsetBytes() const { return (mFakeSize - mElementCount) / 8; }

public:
    PackedContainer();
    PackedContainer(size_t size);
    PackedContainer(size_t size, const std::vector<unsigned>& frozenBits);
    PackedContainer(char* external, size_t size, const std::vector<unsigned>& frozenBits);
    ~PackedContainer();
    void setSize(size_t newSize) override;
    void insertPackedBits(const void* pData) override;
    void insertPackedInformationBits(const void* pData) override;
    void insertCharBits(const void* pData) override;
    void insertLlr(const float* pLlr) override;
    void getPackedBits(void* pData) override;
    void getPackedInformationBits(void* pData) override;
    void resetFrozenBits() override;
    void getFloatBits(float* pData) override;

    /* dummies, as in the reference */
    void insertLlr(const char* pLlr) override;
    void getSoftBits(void* pData) override;
    void getSoftInformation(void* pData) override;

    char* data();
};

} // namespace PolarCode

#endif
