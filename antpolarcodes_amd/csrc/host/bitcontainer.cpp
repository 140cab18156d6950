// bitcontainer.cpp -- the reference's BitContainer family (bitcontainer.cpp of
// david13pod/antPolarCodes) restated in scalar C++ for the host side of this build.
// Every conversion follows the reference's bit/byte semantics; the reference's AVX2
// gathers and movemasks reduce to the MSB-first loops below.  See
// include/polarcode/bitcontainer.h.
#include <polarcode/bitcontainer.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>

namespace PolarCode {

namespace {

constexpr size_t kBitsPerVector = 256;  // BITSPERVECTOR (AVX2)
constexpr size_t kBytesPerVector = 32;  // BYTESPERVECTOR

void* aligned_alloc_or_throw(size_t bytes)
{
    void* p = nullptr;
    if (posix_memalign(&p, 32, std::max<size_t>(bytes, 32)) != 0 || !p)
        throw std::bad_alloc();
    std::memset(p, 0, std::max<size_t>(bytes, 32));
    return p;
}

uint32_t fbits(float f)
{
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

float ffrom(uint32_t u)
{
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}

// convertFtoC (bitcontainer.cpp:27-39): fmin(fmax(x, -128), 127), round() half away from 0
char convert_small(float x)
{
    x = std::fmin(std::fmax(x, -128.0f), 127.0f);
    return static_cast<char>(static_cast<int>(std::round(x)));
}

// vectorizedFtoC (bitcontainer.cpp:449-466): MAXPS(x, -128) (NaN -> -128), MINPS(., 127),
// round to nearest even
char convert_mid(float x)
{
    float t = x > -128.0f ? x : -128.0f;
    t = t < 127.0f ? t : 127.0f;
    return static_cast<char>(static_cast<int>(std::nearbyint(t)));
}

// convert_f32_to_int8_large (bitcontainer.cpp:468-503): cvtps_epi32 (nearest even; NaN and
// out-of-range -> INT_MIN), packs_epi32, packs_epi16 (both saturating)
char convert_large(float x)
{
    if (!(x < 2147483648.0f) || x < -2147483648.0f)
        return static_cast<char>(-128);
    const float r = std::nearbyint(x);
    if (r <= -128.0f)
        return static_cast<char>(-128);
    if (r >= 127.0f)
        return static_cast<char>(127);
    return static_cast<char>(static_cast<int>(r));
}

} // namespace

// ============================================================== BitContainer
BitContainer::BitContainer() : mElementCount(0), mFrozenBits(), mInformationBitCount(0), mLUT(nullptr) {}

BitContainer::BitContainer(size_t size)
    : mElementCount(size), mFrozenBits(), mInformationBitCount((unsigned)size), mLUT(nullptr)
{
}

BitContainer::BitContainer(size_t size, const std::vector<unsigned>& frozenBits)
    : mElementCount(size), mFrozenBits(frozenBits.begin(), frozenBits.end()),
      mInformationBitCount((unsigned)(size - frozenBits.size())), mLUT(nullptr)
{
    calculateLUT();
}

BitContainer::~BitContainer() { clear(); }

void BitContainer::clear()
{
    mFrozenBits.clear();
    mInformationBitCount = (unsigned)mElementCount;
    delete[] mLUT;
    mLUT = nullptr;
}

// the information positions in ascending order (bitcontainer.cpp:68-84)
void BitContainer::calculateLUT()
{
    mLUT = new unsigned[std::max(mInformationBitCount, 8u)]();
    unsigned n = 0;
    size_t f = 0;
    for (unsigned i = 0; i < mElementCount; ++i) {
        if (f < mFrozenBits.size() && mFrozenBits[f] <= i)
            ++f;
        else
            mLUT[n++] = i;
    }
}

size_t BitContainer::size() { return mElementCount; }

void BitContainer::setFrozenBits(const std::vector<unsigned>& frozenBits)
{
    clear();
    mFrozenBits.assign(frozenBits.begin(), frozenBits.end());
    mInformationBitCount = (unsigned)(mElementCount - mFrozenBits.size());
    calculateLUT();
}

// ============================================================== FloatContainer
FloatContainer::FloatContainer() : mData(nullptr), mDataIsExternal(false) {}

FloatContainer::FloatContainer(size_t size) : BitContainer(size), mData(nullptr), mDataIsExternal(false)
{
    setSize(size);
}

FloatContainer::FloatContainer(float* external, size_t size)
    : BitContainer(size), mData(external), mDataIsExternal(true)
{
}

FloatContainer::FloatContainer(size_t size, const std::vector<unsigned>& frozenBits)
    : BitContainer(size, frozenBits), mData(nullptr), mDataIsExternal(false)
{
    setSize(size);
}

FloatContainer::~FloatContainer()
{
    if (!mDataIsExternal)
        std::free(mData);
}

// (the reference asserts newSize % 8 == 0 in debug builds; the GPU decoders also take the
// reference's small codes, N = 2 and 4, so the storage is rounded up instead)
void FloatContainer::setSize(size_t newSize)
{
    mElementCount = newSize;
    if (!mDataIsExternal)
        std::free(mData);
    mDataIsExternal = false;
    mData = static_cast<float*>(aligned_alloc_or_throw(4 * mElementCount));
}

void FloatContainer::insertPackedBits(const void* pData)
{
    const unsigned char* c = static_cast<const unsigned char*>(pData);
    for (size_t i = 0; i < mElementCount / 8 * 8; ++i)
        mData[i] = ffrom(((c[i / 8] >> (7 - i % 8)) & 1u) << 31);
}

void FloatContainer::insertPackedInformationBits(const void* pData)
{
    const unsigned char* c = static_cast<const unsigned char*>(pData);
    std::memset(mData, 0, mElementCount * 4);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        mData[mLUT[j]] = ffrom(((c[j / 8] >> (7 - j % 8)) & 1u) << 31);
}

void FloatContainer::insertCharBits(const void* apData)
{
    // the reference stores the (identity-)converted byte sign-extended into the float word
    const char* c = static_cast<const char*>(apData);
    for (size_t i = 0; i < mElementCount; ++i)
        mData[i] = ffrom(static_cast<uint32_t>(static_cast<int>(convert_small(static_cast<float>(c[i])))));
}

void FloatContainer::insertLlr(const float* pLlr) { std::memcpy(mData, pLlr, 4 * mElementCount); }

void FloatContainer::insertLlr(const char* pLlr)
{
    for (size_t i = 0; i < mElementCount; ++i)
        mData[i] = static_cast<float>(pLlr[i]);
}

void FloatContainer::getPackedBits(void* pData)
{
    // (iBit >> (24 + bit)) truncated to a byte: the whole top byte of the word for bit 0,
    // as the reference does -- exact for +-0.0 bits (bitcontainer.cpp:209-223)
    unsigned char* c = static_cast<unsigned char*>(pData);
    for (size_t b = 0; b < mElementCount / 8; ++b) {
        unsigned char v = 0;
        for (unsigned k = 0; k < 8; ++k)
            v |= static_cast<unsigned char>(fbits(mData[8 * b + k]) >> (24 + k));
        c[b] = v;
    }
}

void FloatContainer::getPackedInformationBits(void* pData)
{
    unsigned char* c = static_cast<unsigned char*>(pData);
    std::memset(c, 0, (mInformationBitCount + 7) / 8);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        c[j / 8] |= static_cast<unsigned char>((fbits(mData[mLUT[j]]) >> 31) << (7 - j % 8));
}

void FloatContainer::getSoftBits(void* pData) { std::memcpy(pData, mData, mElementCount * sizeof(float)); }

void FloatContainer::getFloatBits(float* pData)
{
    for (size_t i = 0; i < mElementCount; ++i)
        pData[i] = ffrom(fbits(mData[i]) & 0x80000000u);
}

void FloatContainer::getSoftInformation(void* pData)
{
    float* f = static_cast<float*>(pData);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        f[j] = mData[mLUT[j]];
}

void FloatContainer::resetFrozenBits()
{
    for (unsigned i : mFrozenBits)
        mData[i] = 0.0f;
}

float* FloatContainer::data() { return mData; }

// ============================================================== CharContainer
CharContainer::CharContainer() : mData(nullptr), mDataIsExternal(false) {}

CharContainer::CharContainer(size_t size) : BitContainer(size), mData(nullptr), mDataIsExternal(false)
{
    setSize(size);
}

CharContainer::CharContainer(char* external, size_t size) : BitContainer(size), mData(external), mDataIsExternal(true)
{
}

CharContainer::CharContainer(size_t size, const std::vector<unsigned>& frozenBits)
    : BitContainer(size, frozenBits), mData(nullptr), mDataIsExternal(false)
{
    setSize(size);
}

CharContainer::~CharContainer()
{
    if (!mDataIsExternal)
        std::free(mData);
}

void CharContainer::setSize(size_t newSize)
{
    mElementCount = newSize;
    if (!mDataIsExternal)
        std::free(mData);
    mDataIsExternal = false;
    mData = static_cast<char*>(aligned_alloc_or_throw(std::max(kBytesPerVector, mElementCount)));
}

void CharContainer::insertPackedBits(const void* pData)
{
    // 0 -> 127, 1 -> 128 (-128)
    const unsigned char* c = static_cast<const unsigned char*>(pData);
    for (size_t i = 0; i < mElementCount / 8 * 8; ++i)
        mData[i] = static_cast<char>(127 + ((c[i / 8] >> (7 - i % 8)) & 1u));
}

void CharContainer::insertPackedInformationBits(const void* pData)
{
    const unsigned char* c = static_cast<const unsigned char*>(pData);
    std::memset(mData, 0, mElementCount);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        mData[mLUT[j]] = static_cast<char>(127 + ((c[j / 8] >> (7 - j % 8)) & 1u));
}

void CharContainer::insertCharBits(const void* pData) { std::memcpy(mData, pData, mElementCount); }

void CharContainer::insertLlr(const float* pLlr)
{
    for (size_t i = 0; i < mElementCount; ++i)
        mData[i] = mElementCount >= 32 ? convert_large(pLlr[i])
                 : mElementCount >= 8  ? convert_mid(pLlr[i])
                                       : convert_small(pLlr[i]);
}

void CharContainer::insertLlr(const char* pLlr) { std::memcpy(mData, pLlr, mElementCount); }

void CharContainer::getPackedBits(void* pData)
{
    const unsigned char* u = reinterpret_cast<const unsigned char*>(mData);
    unsigned char* c = static_cast<unsigned char*>(pData);
    for (size_t b = 0; b < mElementCount / 8; ++b) {
        unsigned char v = 0;
        for (unsigned k = 0; k < 8; ++k)
            v |= static_cast<unsigned char>((u[8 * b + k] & 0x80u) >> k);
        c[b] = v;
    }
}

void CharContainer::getPackedInformationBits(void* pData)
{
    const unsigned char* u = reinterpret_cast<const unsigned char*>(mData);
    unsigned char* c = static_cast<unsigned char*>(pData);
    std::memset(c, 0, (mInformationBitCount + 7) / 8);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        c[j / 8] |= static_cast<unsigned char>((u[mLUT[j]] & 0x80u) >> (j % 8));
}

void CharContainer::getSoftBits(void* pData) { std::memcpy(pData, mData, mElementCount); }

void CharContainer::getFloatBits(float* pData)
{
    const unsigned char* u = reinterpret_cast<const unsigned char*>(mData);
    for (size_t i = 0; i < mElementCount; ++i)
        pData[i] = ffrom(static_cast<uint32_t>(u[i] & 0x80u) << 24);
}

void CharContainer::getSoftInformation(void* pData)
{
    char* c = static_cast<char*>(pData);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        c[j] = mData[mLUT[j]];
}

void CharContainer::resetFrozenBits()
{
    for (unsigned i : mFrozenBits)
        mData[i] = 0;
}

char* CharContainer::data() { return mData; }

// ============================================================== PackedContainer
PackedContainer::PackedContainer() : mData(nullptr), mInformationMask(nullptr), mFakeSize(0), mDataIsExternal(false)
{
}

PackedContainer::PackedContainer(size_t size)
    : BitContainer(size), mData(nullptr), mInformationMask(nullptr), mFakeSize(0), mDataIsExternal(false)
{
    setSize(size);
}

PackedContainer::PackedContainer(size_t size, const std::vector<unsigned>& frozenBits)
    : BitContainer(size, frozenBits), mData(nullptr), mInformationMask(nullptr), mFakeSize(0), mDataIsExternal(false)
{
    setSize(size);
}

PackedContainer::PackedContainer(char* external, size_t size, const std::vector<unsigned>& frozenBits)
    : BitContainer(size, frozenBits), mData(external), mInformationMask(nullptr),
      mFakeSize(std::max(kBitsPerVector, size)), mDataIsExternal(true)
{
    buildInformationMask();
}

PackedContainer::~PackedContainer()
{
    if (!mDataIsExternal)
        std::free(mData);
    delete[] mInformationMask;
}

void PackedContainer::setSize(size_t newSize)
{
    mElementCount = newSize;
    mFakeSize = std::max(kBitsPerVector, mElementCount);
    if (!mDataIsExternal)
        std::free(mData);
    mDataIsExternal = false;
    delete[] mInformationMask;
    mInformationMask = nullptr;
    mData = static_cast<char*>(aligned_alloc_or_throw(mFakeSize / 8));
    buildInformationMask();
}

// The reference's 64-bit word masks (bitcontainer.cpp:671-702) as bytes: whole 64-bit
// words in front of the code are cleared, every other bit kept except the frozen ones.
void PackedContainer::buildInformationMask()
{
    const size_t bytes = mFakeSize / 8;
    delete[] mInformationMask;
    mInformationMask = new unsigned long[bytes / 8]();
    unsigned char* m = reinterpret_cast<unsigned char*>(mInformationMask);
    const size_t offsetBits = mFakeSize - mElementCount;
    const size_t begin = offsetBits >= 64 ? offsetBits / 64 : 0;
    for (size_t b = 0; b < bytes; ++b)
        m[b] = b < begin * 8 ? 0x00 : 0xFF;
    for (unsigned f : mFrozenBits)
        if (f < mElementCount)
            m[offsetBytes() + f / 8] &= static_cast<unsigned char>(~(0x80u >> (f % 8)));
}

void PackedContainer::insertPackedBits(const void* pData)
{
    const size_t nBytes = mElementCount / 8;
    if (nBytes < mFakeSize / 8)
        std::memcpy(mData + (kBytesPerVector - nBytes), pData, nBytes);
    else
        std::memcpy(mData, pData, nBytes);
}

void PackedContainer::insertPackedInformationBits(const void* pData)
{
    const unsigned char* c = static_cast<const unsigned char*>(pData);
    unsigned char* u = reinterpret_cast<unsigned char*>(mData);
    std::memset(mData, 0, mFakeSize / 8);
    u += offsetBytes();
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        if ((c[j / 8] >> (7 - j % 8)) & 1u)
            u[mLUT[j] / 8] |= static_cast<unsigned char>(0x80u >> (mLUT[j] % 8));
}

void PackedContainer::insertCharBits(const void* pData)
{
    // at the buffer's start, without the N < 256 offset, as the reference
    const unsigned char* in = static_cast<const unsigned char*>(pData);
    unsigned char* out = reinterpret_cast<unsigned char*>(mData);
    for (size_t b = 0; b < mElementCount / 8; ++b) {
        unsigned char v = 0;
        for (unsigned k = 0; k < 8; ++k)
            v |= static_cast<unsigned char>((in[8 * b + k] & 0x80u) >> k);
        out[b] = v;
    }
}

void PackedContainer::insertLlr(const float* pData)
{
    unsigned char* out = reinterpret_cast<unsigned char*>(mData) + offsetBytes();
    for (size_t b = 0; b < mElementCount / 8; ++b) {
        unsigned char v = 0;
        for (unsigned k = 0; k < 8; ++k)
            v |= static_cast<unsigned char>((fbits(pData[8 * b + k]) & 0x80000000u) >> (k + 24));
        out[b] = v;
    }
}

void PackedContainer::getPackedBits(void* pData) { std::memcpy(pData, mData + offsetBytes(), mElementCount / 8); }

void PackedContainer::resetFrozenBits()
{
    const unsigned char* m = reinterpret_cast<const unsigned char*>(mInformationMask);
    unsigned char* u = reinterpret_cast<unsigned char*>(mData);
    for (size_t b = 0; b < mFakeSize / 8; ++b)
        u[b] &= m[b];
}

char* PackedContainer::data() { return mData; }

void PackedContainer::insertLlr(const char*) {}
void PackedContainer::getSoftBits(void*) {}
void PackedContainer::getSoftInformation(void*) {}

void PackedContainer::getFloatBits(float* pData)
{
    // from the buffer's start, like the reference (no N < 256 offset)
    const unsigned char* u = reinterpret_cast<const unsigned char*>(mData);
    for (size_t i = 0; i < mElementCount; ++i)
        pData[i] = ffrom(static_cast<uint32_t>((u[i / 8] << (i % 8)) & 0x80u) << 24);
}

void PackedContainer::getPackedInformationBits(void* pData)
{
    const unsigned char* u = reinterpret_cast<const unsigned char*>(mData) + offsetBytes();
    unsigned char* c = static_cast<unsigned char*>(pData);
    std::memset(c, 0, (mInformationBitCount + 7) / 8);
    for (unsigned j = 0; j < mInformationBitCount; ++j)
        if ((u[mLUT[j] / 8] >> (7 - mLUT[j] % 8)) & 1u)
            c[j / 8] |= static_cast<unsigned char>(0x80u >> (j % 8));
}

} // namespace PolarCode
