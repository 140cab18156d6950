// polarcode_host.cpp -- host C++ library (libpolarcode_amd.so) mirroring the
// reference's PolarCode::{ErrorDetection, Construction, Encoding, Decoding} API on
// top of the C ABI (include/pcg.h).  No device code here.
#include <polarcode/construction/constructor.h>
#include <polarcode/decoding/decoder.h>
#include <polarcode/encoding/butterfly_fip_packed.h>
#include <polarcode/encoding/encoder.h>
#include <polarcode/errordetection/errordetector.h>
#include <polarcode/puncturer.h>

#include "../crc_host.hpp"
#include <pcg.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>

namespace PolarCode {

// =============================================================== ErrorDetection
namespace ErrorDetection {

Dummy globalDummyDetector;

void Crc::generate(void* data, int bytes) { pcg::crc_generate((int)mBits, static_cast<uint8_t*>(data), bytes); }

bool Crc::check(void* data, int bytes) { return pcg::crc_check((int)mBits, static_cast<uint8_t*>(data), bytes); }

int Crc::multiCheck(void** data, int nArrays, int nBytes)
{
    for (int a = 0; a < nArrays; ++a)
        if (check(data[a], nBytes))
            return a;
    return -1;
}

Detector* create(unsigned size, std::string type)
{
    std::transform(type.begin(), type.end(), type.begin(), [](unsigned char c) { return std::tolower(c); });
    if (type.find("crc") != std::string::npos) {
        switch (size) {
        case 0:
            return new Dummy();
        case 8:
            return new CRC8();
        case 11:
            return new CRC11();
        case 16:
            return new CRC16();
        case 32:
            return new CRC32();
        default:
            throw std::logic_error("CRC INVALID SIZE!");
        }
    }
    if (type.find("cmac") != std::string::npos)
        throw std::logic_error("CMAC detectors are not part of this build");
    throw std::runtime_error("Unknown Error detector requested!");
}

int gpuKind(Detector* d)
{
    if (!d)
        return 0;
    const std::string t = d->getType();
    if (t == "DUMMY")
        return 0;
    if (t == "CRC") {
        const unsigned b = d->getCheckBitCount();
        if (b == 0 || b == 8 || b == 11 || b == 16 || b == 32)
            return (int)b;
    }
    return -1;
}

} // namespace ErrorDetection

// =============================================================== Construction
namespace Construction {

namespace {
const unsigned short kNrRank[1024] = {
#include "nr_reliability.inc"
};

std::string lower(std::string t)
{
    std::transform(t.begin(), t.end(), t.begin(), [](unsigned char c) { return std::tolower(c); });
    return t;
}

void check_lengths(size_t N, size_t K)
{
    if (N < K) // fiveGList.cpp:30-34, betaexpansion.cpp:47-51
        throw std::invalid_argument("Invalid polar code(" + std::to_string(N) + ", " + std::to_string(K) + ")");
}
} // namespace

void Constructor::setBlockLength(size_t newBlockLength)
{
    const size_t test = newBlockLength ? (size_t)1 << (size_t)std::log2((double)newBlockLength) : 0;
    if (test != newBlockLength) // constructor.cpp:25-32
        throw std::invalid_argument("new blockLength is not a power of 2!");
    mBlockLength = newBlockLength;
}

Bhattacharrya::Bhattacharrya(size_t N, size_t K, float designSnr)
{
    setBlockLength(N);
    setInformationLength(K);
    setDesignSnr(designSnr);
}

std::vector<unsigned> Bhattacharrya::construct()
{
    const size_t N = mBlockLength, K = mInformationLength;
    if (K > N)
        throw std::invalid_argument("information length exceeds block length");
    // initial parameter in float (bhattacharrya.cpp:39-44), recursion in double (:66-80)
    const float lin = (float)std::pow(10.0, mDesignSnr / 10.0);
    const float init = (float)std::exp(-2.0 * lin * K / N);
    std::vector<double> z(N);
    z[0] = init;
    for (int stage = (int)std::log2((double)N) - 1; stage >= 0; --stage) {
        const size_t B = (size_t)1 << stage;
        for (size_t j = 0; j < N; j += 2 * B) {
            const double T = z[j];
            z[j + B] = T * T;
            z[j] = 2 * T - z[j + B];
        }
    }
    // trackingSorter::stableSortDescending (arrayfuncs.cpp:93-107)
    std::vector<unsigned> perm(N);
    for (size_t i = 0; i < N; ++i)
        perm[i] = (unsigned)i;
    std::stable_sort(perm.begin(), perm.end(), [&](unsigned a, unsigned b) { return z[a] > z[b]; });
    std::vector<unsigned> f(perm.begin(), perm.begin() + (N - K));
    std::sort(f.begin(), f.end());
    return f;
}

FiveGList::FiveGList(size_t N, size_t K)
{
    if (N > 1024) // fiveGList.cpp:21-23
        throw std::invalid_argument("5G standard does not allow for block size N > 1024!");
    setBlockLength(N);
    setInformationLength(K);
}

std::vector<unsigned> FiveGList::construct()
{
    check_lengths(mBlockLength, mInformationLength);
    // the first N-K entries of the 1024-entry sequence, ascending (fiveGList.cpp:35-39):
    // exactly the indices whose reliability rank is < N-K
    const unsigned nf = (unsigned)(mBlockLength - mInformationLength);
    std::vector<unsigned> f;
    f.reserve(nf);
    for (unsigned i = 0; i < 1024; ++i)
        if (kNrRank[i] < nf)
            f.push_back(i);
    return f;
}

BetaExpansion::BetaExpansion(size_t N, size_t K)
{
    setBlockLength(N);
    setInformationLength(K);
}

std::vector<unsigned> BetaExpansion::construct()
{
    check_lengths(mBlockLength, mInformationLength);
    const unsigned n = (unsigned)std::log2((double)mBlockLength);
    const double beta = std::pow(2.0, 1.0 / 4.0);
    std::vector<double> wj(n), w(mBlockLength);
    for (unsigned j = 0; j < n; ++j)
        wj[j] = std::pow(beta, (double)j);
    for (size_t i = 0; i < mBlockLength; ++i) {
        double acc = 0.0;
        for (unsigned j = 0; j < n; ++j)
            acc += wj[j] * ((i >> j) & 1u);
        w[i] = acc;
    }
    // argsort ascending with the same std::sort call shape (betaexpansion.cpp:19-31)
    std::vector<size_t> idx(mBlockLength);
    for (size_t i = 0; i < mBlockLength; ++i)
        idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&w](int l, int r) -> bool { return w[l] < w[r]; });
    std::vector<unsigned> f(idx.begin(), idx.begin() + (mBlockLength - mInformationLength));
    std::sort(f.begin(), f.end());
    return f;
}

std::vector<unsigned> frozen_bits(const int blockLength,
                                  const int infoLength,
                                  const float designSNR,
                                  const std::string& constructor_type)
{
    const std::string t = lower(constructor_type);
    if (t.find("be") != std::string::npos)
        return BetaExpansion((size_t)blockLength, (size_t)infoLength, designSNR).construct();
    if (t.find("5g") != std::string::npos)
        return FiveGList((size_t)blockLength, (size_t)infoLength, designSNR).construct();
    return Bhattacharrya((size_t)blockLength, (size_t)infoLength, designSNR).construct();
}

} // namespace Construction

// =============================================================== Puncturer
size_t round_up_power_of_two(size_t value)
{
    // the 32-bit bit trick, deliberately unextended (puncturer.cpp:23-33)
    value--;
    value |= value >> 1;
    value |= value >> 2;
    value |= value >> 4;
    value |= value >> 8;
    value |= value >> 16;
    return value + 1;
}

std::vector<unsigned> inverse_set_difference(size_t blockLength, std::vector<unsigned> positions)
{
    // the std::set_difference merge over iota(blockLength) and `positions`
    std::vector<unsigned> out;
    size_t j = 0;
    for (unsigned v = 0; v < blockLength;) {
        if (j == positions.size()) {
            out.push_back(v++);
        } else if (v < positions[j]) {
            out.push_back(v++);
        } else {
            if (!(positions[j] < v))
                ++v;
            ++j;
        }
    }
    return out;
}

Puncturer::Puncturer(const size_t blockLength, const std::vector<unsigned> frozenBitPositions)
    : mBlockLength(blockLength)
{
    mParentBlockLength = round_up_power_of_two(mBlockLength);
    const size_t np = mParentBlockLength - mBlockLength;
    if (np > frozenBitPositions.size())
        throw std::out_of_range("Number of required puncturing positions exceeds frozen bit positions!");
    mOutputPositions = inverse_set_difference(
        mParentBlockLength, std::vector<unsigned>(frozenBitPositions.begin(), frozenBitPositions.begin() + np));
}

Puncturer::~Puncturer() {}

void Puncturer::puncturePacked(unsigned char* pOutput, const unsigned char* pInput)
{
    const size_t bytes = mBlockLength / 8;
    for (size_t b = 0; b < bytes; ++b) {
        unsigned o = 0;
        for (unsigned i = 0; i < 8; ++i) {
            const unsigned p = mOutputPositions[8 * b + i];
            o |= ((pInput[p / 8] >> (7 - p % 8)) & 1u) << (7 - i);
        }
        pOutput[b] = (unsigned char)o;
    }
}

// =============================================================== Encoding
namespace Encoding {

Encoder::Encoder()
    : mEncoderDuration(0), mErrorDetector(&ErrorDetection::globalDummyDetector), mBlockLength(0), mSystematic(true),
      mCodewordReady(false), xmInputData(nullptr), mBitContainer(nullptr)
{
}

Encoder::~Encoder() { delete mBitContainer; }

size_t Encoder::blockLength() { return mBlockLength; }

void Encoder::setErrorDetection(ErrorDetection::Detector* pDetector) { mErrorDetector = pDetector; }

void Encoder::setSystematic(bool sys) { mSystematic = sys; }

bool Encoder::isSystematic() { return mSystematic; }

void Encoder::setInformation(void* pData) { xmInputData = static_cast<unsigned char*>(pData); }

void Encoder::getInformation(void* pData) { mBitContainer->getPackedInformationBits(pData); }

void Encoder::setCodeword(void* pData)
{
    xmInputData = static_cast<unsigned char*>(pData);
    mBitContainer->insertPackedBits(pData);
    mCodewordReady = true;
}

void Encoder::setCharCodeword(void* cData)
{
    mBitContainer->insertCharBits(cData);
    mCodewordReady = true;
}

void Encoder::setFloatCodeword(void* fData)
{
    mBitContainer->insertLlr(static_cast<float*>(fData));
    mCodewordReady = true;
}

void Encoder::getEncodedData(void* pData) { mBitContainer->getPackedBits(pData); }

void Encoder::clearFrozenBits() { mBitContainer->resetFrozenBits(); }

void Encoder::encode_vector(void* pInfo, void* pCode)
{
    const auto t0 = std::chrono::steady_clock::now();
    setInformation(pInfo);
    encode();
    getEncodedData(pCode);
    mEncoderDuration =
        (size_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

UndefinedEncoder::UndefinedEncoder() {}

UndefinedEncoder::~UndefinedEncoder() {}

void UndefinedEncoder::initialize(size_t, const std::vector<unsigned>&) {}

void UndefinedEncoder::encode() { std::fprintf(stderr, "Call to UndefinedEncoder::encode()!\n"); }

ButterflyFipPacked::ButterflyFipPacked() {}

ButterflyFipPacked::ButterflyFipPacked(size_t blockLength) { initialize(blockLength, {}); }

ButterflyFipPacked::ButterflyFipPacked(size_t blockLength, const std::vector<unsigned>& frozenBits)
{
    initialize(blockLength, frozenBits);
}

ButterflyFipPacked::~ButterflyFipPacked() {}

void ButterflyFipPacked::initialize(size_t blockLength, const std::vector<unsigned>& frozenBits)
{
    mBlockLength = blockLength;
    mFrozenBits.assign(frozenBits.begin(), frozenBits.end());
    delete mBitContainer;
    mBitContainer = new PackedContainer(mBlockLength, mFrozenBits);
}

// butterfly_fip_packed.cpp:45-59: the detector's check bits into the caller's bytes, the
// bits into the container, transform; systematic: clear the frozen bits, transform again
void ButterflyFipPacked::encode()
{
    if (!mCodewordReady) {
        mErrorDetector->generate(xmInputData, (int)((mBlockLength - mFrozenBits.size()) / 8));
        mBitContainer->insertPackedInformationBits(xmInputData);
    }
    transform();
    if (mSystematic) {
        mBitContainer->resetFrozenBits();
        transform();
    }
    mCodewordReady = false;
}

// x[i] ^= x[i + 2^s] for every i with bit s clear, all stages (butterfly_fip.cpp:15-63),
// over the code's packed MSB-first bytes (the end of the 256-bit buffer when N < 256)
void ButterflyFipPacked::transform()
{
    const size_t N = mBlockLength;
    auto* pc = static_cast<PackedContainer*>(mBitContainer);
    unsigned char* x = reinterpret_cast<unsigned char*>(pc->data()) + (std::max<size_t>(256, N) - N) / 8;
    static const unsigned char kMask[3] = { 0xAA, 0xCC, 0xF0 }; // positions i with bit s clear, s < 3
    const size_t bytes = N / 8;
    for (size_t B = 1; B < N; B <<= 1) {
        if (B < 8) {
            const unsigned s = (unsigned)__builtin_ctzll(B);
            for (size_t j = 0; j < bytes; ++j)
                x[j] ^= (unsigned char)((x[j] << B) & kMask[s]);
        } else {
            const size_t b = B / 8;
            for (size_t j = 0; j < bytes; j += 2 * b)
                for (size_t k = j; k < j + b; ++k)
                    x[k] ^= x[k + b];
        }
    }
}

} // namespace Encoding

// =============================================================== Decoding
namespace Decoding {

Decoder::Decoder()
    : mDecoderDuration(0), mErrorDetector(&ErrorDetection::globalDummyDetector), mBlockLength(0), mSystematic(true),
      mLlrContainer(nullptr), mBitContainer(nullptr), mOutputContainer(nullptr), mFrozenBits(),
      mExternalContainers(false)
{
}

Decoder::~Decoder()
{
    if (!mExternalContainers) {
        delete mLlrContainer;
        delete mBitContainer;
        delete[] mOutputContainer;
    }
}

void Decoder::initialize(size_t blockLength, const std::vector<unsigned>& frozenBits)
{
    mBlockLength = blockLength;
    mFrozenBits.assign(frozenBits.begin(), frozenBits.end());
}

size_t Decoder::blockLength() { return mBlockLength; }

size_t Decoder::infoLength() { return mBlockLength - mFrozenBits.size(); }

BitContainer* Decoder::inputContainer() { return mLlrContainer; }

BitContainer* Decoder::outputContainer() { return mBitContainer; }

unsigned char* Decoder::packedOutput() { return mOutputContainer; }

void Decoder::setSystematic(bool sys) { mSystematic = sys; }

bool Decoder::isSystematic() { return mSystematic; }

void Decoder::setErrorDetection(ErrorDetection::Detector* pDetector) { mErrorDetector = pDetector; }

void Decoder::setSignal(const float* pLlr) { mLlrContainer->insertLlr(pLlr); }

void Decoder::setSignal(const char* pLlr) { mLlrContainer->insertLlr(pLlr); }

void Decoder::getDecodedInformationBits(void* pData)
{
    std::memcpy(pData, mOutputContainer, (mBlockLength - mFrozenBits.size() + 7) / 8);
}

void Decoder::getSoftCodeword(void* pData) { mBitContainer->getSoftBits(pData); }

void Decoder::getSoftInformation(void* pData) { mBitContainer->getSoftInformation(pData); }

bool Decoder::decodeBatch(const float* llr, size_t F, uint8_t* info, uint8_t* ok, float*)
{
    const size_t kb = (infoLength() + 7) / 8;
    bool all = true;
    for (size_t f = 0; f < F; ++f) {
        const bool r = decode_vector(llr + f * mBlockLength, info + f * kb);
        if (ok)
            ok[f] = r ? 1 : 0;
        all = all && r;
    }
    return all;
}

void Decoder::decodeBatchDevice(const float*, size_t, uint8_t*, uint8_t*, float*, void*)
{
    throw std::logic_error("decodeBatchDevice needs a GPU decoder");
}

bool Decoder::decodeBatchI8(const int8_t* llr, size_t F, uint8_t* info, uint8_t* ok, float*)
{
    const size_t kb = (infoLength() + 7) / 8;
    bool all = true;
    for (size_t f = 0; f < F; ++f) {
        const bool r = decode_vector(reinterpret_cast<const char*>(llr) + f * mBlockLength, info + f * kb);
        if (ok)
            ok[f] = r ? 1 : 0;
        all = all && r;
    }
    return all;
}

bool Decoder::decode_vector(const float* pLlr, void* pData)
{
    const auto t0 = std::chrono::steady_clock::now();
    setSignal(pLlr);
    const bool r = decode();
    getDecodedInformationBits(pData);
    mDecoderDuration =
        (size_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    return r;
}

bool Decoder::decode_vector(const char* pLlr, void* pData)
{
    const auto t0 = std::chrono::steady_clock::now();
    setSignal(pLlr);
    const bool r = decode();
    getDecodedInformationBits(pData);
    mDecoderDuration =
        (size_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    return r;
}

UndefinedDecoder::UndefinedDecoder() {}

UndefinedDecoder::~UndefinedDecoder() {}

bool UndefinedDecoder::decode()
{
    std::fprintf(stderr, "Call to UndefinedDecoder::decode()!\n");
    return false;
}

// Soft accessors of the GPU decoders' output container.  Fast-SSC float decoders (N <= 16384)
// hold the reference's soft codeword word for word; every other GPU decoder holds the selected
// path's signed hard decisions (+0.0 / -0.0, or the char bits 127 / -128).  Only the signs of the
// reference's list / 8-bit "bit" buffers are observable (scl_avx_float.cpp:711-750 copies the
// selected path's Bit(path, dataStage) into mBitContainer; decoder.cpp:147-151 returns it), so the
// signs are the reference's.
void DecodedFloatContainer::getSoftBits(void* pData) { FloatContainer::getSoftBits(pData); }

void DecodedFloatContainer::getSoftInformation(void* pData) { FloatContainer::getSoftInformation(pData); }

void DecodedCharContainer::getSoftBits(void* pData) { CharContainer::getSoftBits(pData); }

void DecodedCharContainer::getSoftInformation(void* pData) { CharContainer::getSoftInformation(pData); }

static void throw_pcg(int rc)
{
    const std::string msg = pcg_last_error();
    if (rc == PCG_E_FROZEN)
        throw std::invalid_argument(msg);
    if (rc == PCG_E_ARG)
        throw std::logic_error(msg);
    throw std::runtime_error("pcg error " + std::to_string(rc) + ": " + msg);
}

GpuDecoder::GpuDecoder(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int device)
    : mListSize(listSize), mDevice(device), mStageDetector(mErrorDetector)
{
    initialize(blockLength, frozenBits);
}

GpuDecoder::~GpuDecoder() { releasePlan(); }

void GpuDecoder::releasePlan()
{
    if (mPlan)
        pcg_plan_destroy(mPlan);
    mPlan = nullptr;
}

// the reference decoders' containers (fastssc_avx_float.cpp:933-937, scl_avx_float.cpp:691-693,
// fastssc_fip_char.cpp:607-613, scl_fip_char.cpp:796-798): float or char input, an output
// container, (K+7)/8 packed output bytes
void GpuDecoder::setupContainers()
{
    if (!mExternalContainers) {
        delete mLlrContainer;
        delete mBitContainer;
        delete[] mOutputContainer;
    }
    mExternalContainers = false;
    if (mFixed) {
        mLlrContainer = new CharContainer(mBlockLength, mFrozenBits);
        mBitContainer = new DecodedCharContainer(mBlockLength, mFrozenBits);
    } else {
        mLlrContainer = new FloatContainer(mBlockLength, mFrozenBits);
        mBitContainer = new DecodedFloatContainer(mBlockLength, mFrozenBits);
    }
    mOutputContainer = new unsigned char[(mBlockLength - mFrozenBits.size() + 7) / 8 + 1]();
}

void GpuDecoder::initialize(size_t blockLength, const std::vector<unsigned>& frozenBits)
{
    Decoder::initialize(blockLength, frozenBits);
    releasePlan();
    // validate (and classify) now so invalid codes fail at construction like the reference
    pcg_plan* probe = nullptr;
    int rc = (mFixed ? pcg_plan_create_char : pcg_plan_create)(&probe, (uint32_t)blockLength, (uint32_t)mListSize,
                                                                 mFrozenBits.data(), (uint32_t)mFrozenBits.size(),
                                                                 1, 0, -1);
    if (rc != 0)
        throw_pcg(rc);
    pcg_plan_destroy(probe);
    if (mAdaptive) { // AdaptiveFloat / AdaptiveChar also construct their Fast-SSC decoder
        rc = (mFixed ? pcg_plan_create_char : pcg_plan_create)(&probe, (uint32_t)blockLength, 1, mFrozenBits.data(),
                                                               (uint32_t)mFrozenBits.size(), 1, 0, -1);
        if (rc != 0)
            throw_pcg(rc);
        pcg_plan_destroy(probe);
    }
    setupContainers();
}

void GpuDecoder::setSystematic(bool sys)
{
    mStageSystematic = sys;
    if (!mAdaptive) // AdaptiveFloat::setSystematic sets its stages only (adaptive_float.cpp:47-51)
        mSystematic = sys;
}

void GpuDecoder::setErrorDetection(ErrorDetection::Detector* pDetector)
{
    if (ErrorDetection::gpuKind(pDetector) < 0)
        throw std::logic_error("detector " + pDetector->getType() + " cannot be evaluated on the GPU");
    mStageDetector = pDetector;
    if (!mAdaptive) // AdaptiveFloat::setErrorDetection sets its stages only (adaptive_float.cpp:53-57)
        mErrorDetector = pDetector;
}

void GpuDecoder::ensurePlan()
{
    const int kind = ErrorDetection::gpuKind(mStageDetector);
    if (mPlan && kind == mPlanKind && mStageSystematic == mPlanSys)
        return;
    releasePlan();
    auto create = mAdaptive ? (mFixed ? pcg_plan_create_adaptive_char : pcg_plan_create_adaptive)
                            : (mFixed ? pcg_plan_create_char : pcg_plan_create);
    const int rc = create(&mPlan, (uint32_t)mBlockLength, (uint32_t)mListSize, mFrozenBits.data(),
                          (uint32_t)mFrozenBits.size(), mStageSystematic ? 1 : 0, kind, mDevice);
    if (rc != 0) {
        mPlan = nullptr;
        throw_pcg(rc);
    }
    mPlanKind = kind;
    mPlanSys = mStageSystematic;
}

// The decoded codeword's hard decisions into the output container: every decoder output is
// a codeword, so it is the (systematic or not) encoding of the decoded information bits
// (butterfly_fip_packed.cpp:45-70 on one bit per byte, any N).
void GpuDecoder::fillHardCodeword()
{
    const size_t N = mBlockLength;
    std::vector<uint8_t> x(N, 0), frozen(N, 0);
    for (unsigned f : mFrozenBits)
        frozen[f] = 1;
    for (size_t i = 0, j = 0; i < N; ++i)
        if (!frozen[i]) {
            x[i] = (mOutputContainer[j / 8] >> (7 - j % 8)) & 1u;
            ++j;
        }
    auto transform = [&]() {
        for (size_t B = 1; B < N; B <<= 1)
            for (size_t j = 0; j < N; j += 2 * B)
                for (size_t i = j; i < j + B; ++i)
                    x[i] ^= x[i + B];
    };
    transform();
    if (mStageSystematic) {
        for (size_t i = 0; i < N; ++i)
            if (frozen[i])
                x[i] = 0;
        transform();
    }
    if (auto* fc = dynamic_cast<DecodedFloatContainer*>(mBitContainer)) {
        std::vector<float> bits(N);
        for (size_t i = 0; i < N; ++i)
            bits[i] = x[i] ? -0.0f : 0.0f;
        fc->insertLlr(bits.data());
        fc->setSoft(false);
    } else {
        std::vector<char> bits(N);
        for (size_t i = 0; i < N; ++i)
            bits[i] = static_cast<char>(x[i] ? -128 : 127); // CharContainer::insertPackedBits' format
        mBitContainer->insertCharBits(bits.data());
    }
}

bool GpuDecoder::decode()
{
    // one frame of one reused decoder instance: Fast-SSC float decoders also return the
    // soft codeword (getSoftCodeword); list decoders start from the carried path-0 metric
    // and keep the new one (the reference's PathList never resets mMetric, Q8)
    ensurePlan();
    uint8_t ok = 0;
    int rc;
    bool soft = false;
    if (mListSize <= 1 && !mFixed && !mAdaptive) {
        auto* out = static_cast<DecodedFloatContainer*>(mBitContainer);
        rc = pcg_decode_f32_soft_host(mPlan, static_cast<FloatContainer*>(mLlrContainer)->data(), 1,
                                      mOutputContainer, &ok, out->data());
        if (rc == PCG_E_UNSUPPORTED) // N beyond the soft kernel's LDS: hard decisions only
            rc = pcg_decode_f32_host(mPlan, static_cast<FloatContainer*>(mLlrContainer)->data(), 1,
                                     mOutputContainer, &ok, nullptr);
        else
            soft = rc == 0;
        if (rc != 0)
            throw_pcg(rc);
        out->setSoft(soft);
    } else {
        // (the adaptive decoders' list stage runs only for failed frames: no carry there)
        const bool carry = mListSize > 1 && !mAdaptive;
        std::vector<float> met(mListSize > 1 ? mListSize : 1, 0.0f);
        float* mp = carry ? met.data() : nullptr;
        if (carry && (rc = pcg_plan_set_initial_metric(mPlan, mCarry)) != 0)
            throw_pcg(rc);
        if (mFixed)
            rc = pcg_decode_i8_host(mPlan, reinterpret_cast<const int8_t*>(static_cast<CharContainer*>(
                                               mLlrContainer)->data()), 1, mOutputContainer, &ok, mp);
        else
            rc = pcg_decode_f32_host(mPlan, static_cast<FloatContainer*>(mLlrContainer)->data(), 1,
                                     mOutputContainer, &ok, mp);
        if (carry)
            (void)pcg_plan_set_initial_metric(mPlan, 0.0f); // batches keep fresh-decoder semantics
        if (rc != 0)
            throw_pcg(rc);
        if (carry)
            mCarry = met[0];
    }
    if (!soft)
        fillHardCodeword();
    return ok != 0;
}

bool GpuDecoder::decodeBatch(const float* llr, size_t F, uint8_t* info, uint8_t* ok, float* metrics)
{
    ensurePlan();
    std::vector<uint8_t> okv;
    uint8_t* okp = ok;
    if (!okp) {
        okv.assign(F, 0);
        okp = okv.data();
    }
    const int rc = pcg_decode_f32_host(mPlan, llr, F, info, okp, mListSize > 1 ? metrics : nullptr);
    if (rc != 0)
        throw_pcg(rc);
    for (size_t f = 0; f < F; ++f)
        if (!okp[f])
            return false;
    return true;
}

void GpuDecoder::decodeBatchDevice(const float* llr, size_t F, uint8_t* info, uint8_t* ok, float* metrics,
                                   void* hipStream)
{
    ensurePlan();
    const int rc = pcg_decode_f32(mPlan, llr, F, info, ok, mListSize > 1 ? metrics : nullptr, hipStream);
    if (rc != 0)
        throw_pcg(rc);
}

bool GpuDecoder::decodeBatchI8(const int8_t* llr, size_t F, uint8_t* info, uint8_t* ok, float* metrics)
{
    if (!mFixed) { // float decoders take 8-bit LLRs as floats (FloatContainer::insertLlr(const char*))
        std::vector<float> f((size_t)F * mBlockLength);
        for (size_t i = 0; i < f.size(); ++i)
            f[i] = static_cast<float>(llr[i]);
        return decodeBatch(f.data(), F, info, ok, metrics);
    }
    ensurePlan();
    std::vector<uint8_t> okv;
    uint8_t* okp = ok;
    if (!okp) {
        okv.assign(F, 0);
        okp = okv.data();
    }
    const int rc = pcg_decode_i8_host(mPlan, llr, F, info, okp, mListSize > 1 ? metrics : nullptr);
    if (rc != 0)
        throw_pcg(rc);
    for (size_t f = 0; f < F; ++f)
        if (!okp[f])
            return false;
    return true;
}

void GpuDecoder::decodeBatchDeviceI8(const int8_t* llr, size_t F, uint8_t* info, uint8_t* ok, float* metrics,
                                     void* hipStream)
{
    if (!mFixed)
        throw std::logic_error("int8 device frames need an 8-bit (\"char\") decoder");
    ensurePlan();
    const int rc = pcg_decode_i8(mPlan, llr, F, info, ok, mListSize > 1 ? metrics : nullptr, hipStream);
    if (rc != 0)
        throw_pcg(rc);
}

GpuFastSscChar::GpuFastSscChar(size_t blockLength, const std::vector<unsigned>& frozenBits, int device)
    : GpuDecoder(blockLength, 1, {}, device)
{
    mFixed = true;
    initialize(blockLength, frozenBits);
}

GpuSclChar::GpuSclChar(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int device)
    : GpuDecoder(blockLength, listSize, {}, device)
{
    mFixed = true;
    initialize(blockLength, frozenBits);
}

GpuAdaptiveChar::GpuAdaptiveChar(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                                 int device)
    : GpuDecoder(blockLength, listSize, {}, device)
{
    mAdaptive = true;
    mFixed = true;
    initialize(blockLength, frozenBits);
}

GpuAdaptiveFloat::GpuAdaptiveFloat(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                                   int device)
    : GpuDecoder(blockLength, listSize, {}, device)
{
    mAdaptive = true;
    initialize(blockLength, frozenBits); // validate both stages now (GpuDecoder's ran before mAdaptive)
}

// AdaptiveMixed (adaptive_mixed.cpp:14-78)
GpuAdaptiveMixed::GpuAdaptiveMixed(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits,
                                   int device)
    : mFastDecoder(nullptr), mListDecoder(nullptr), mListSize(listSize)
{
    mBlockLength = blockLength;
    mFrozenBits.assign(frozenBits.begin(), frozenBits.end());
    mExternalContainers = true;
    mFastDecoder = new GpuFastSscChar(mBlockLength, mFrozenBits, device);
    try {
        mListDecoder = new GpuSclFloat(mBlockLength, mListSize, mFrozenBits, device);
    } catch (...) {
        delete mFastDecoder;
        throw;
    }
    // like the reference, no containers of its own: setSignal(const float*) feeds both
    // stages; inputContainer() is null (the non-virtual setSignal(const char*) is not usable)
}

GpuAdaptiveMixed::~GpuAdaptiveMixed()
{
    delete mFastDecoder;
    delete mListDecoder;
}

bool GpuAdaptiveMixed::decode()
{
    bool success = mFastDecoder->decode();
    mOutputContainer = mFastDecoder->packedOutput();
    mBitContainer = mFastDecoder->outputContainer();
    if (!success && mListSize > 1) {
        success = mListDecoder->decode();
        mOutputContainer = mListDecoder->packedOutput();
        mBitContainer = mListDecoder->outputContainer();
    }
    return success;
}

void GpuAdaptiveMixed::setSystematic(bool sys)
{
    mFastDecoder->setSystematic(sys);
    mListDecoder->setSystematic(sys);
}

void GpuAdaptiveMixed::setErrorDetection(ErrorDetection::Detector* pDetector)
{
    mFastDecoder->setErrorDetection(pDetector);
    mListDecoder->setErrorDetection(pDetector);
}

void GpuAdaptiveMixed::setSignal(const float* pLlr)
{
    mFastDecoder->setSignal(pLlr);
    mListDecoder->setSignal(pLlr);
}

bool GpuAdaptiveMixed::decodeBatch(const float* llr, size_t F, uint8_t* info, uint8_t* ok, float*)
{
    const size_t N = mBlockLength, kb = (infoLength() + 7) / 8;
    std::vector<uint8_t> okv(F, 0);
    mFastDecoder->decodeBatch(llr, F, info, okv.data()); // the 8-bit plan quantises (insertLlr)
    std::vector<size_t> bad;
    for (size_t f = 0; f < F; ++f)
        if (!okv[f])
            bad.push_back(f);
    if (!bad.empty() && mListSize > 1) {
        std::vector<float> sub(bad.size() * N);
        for (size_t i = 0; i < bad.size(); ++i)
            std::memcpy(&sub[i * N], llr + bad[i] * N, N * sizeof(float));
        std::vector<uint8_t> si(bad.size() * kb), sk(bad.size());
        mListDecoder->decodeBatch(sub.data(), bad.size(), si.data(), sk.data());
        for (size_t i = 0; i < bad.size(); ++i) {
            std::memcpy(info + bad[i] * kb, &si[i * kb], kb);
            okv[bad[i]] = sk[i];
        }
    }
    bool all = true;
    for (size_t f = 0; f < F; ++f) {
        if (ok)
            ok[f] = okv[f];
        all = all && okv[f];
    }
    return all;
}

Decoder* makeDecoder(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, int impl)
{
    Decoder* dec;
    if (listSize == 1) { // decoder.cpp:60-68: 1 -> float, anything else -> 8-bit
        if (impl == 1)
            dec = new GpuFastSscFloat(blockLength, frozenBits);
        else
            dec = new GpuFastSscChar(blockLength, frozenBits);
    } else { // decoder.cpp:69-83
        switch (impl) {
        case 1:
            dec = new GpuSclFloat(blockLength, listSize, frozenBits);
            break;
        case 2:
            dec = new GpuAdaptiveFloat(blockLength, listSize, frozenBits);
            break;
        case 3:
            throw std::logic_error("decoder implementation 3 (SCAN) is not part of this build");
        default:
            dec = new GpuSclChar(blockLength, listSize, frozenBits);
            break;
        }
    }
    dec->setErrorDetection(new ErrorDetection::CRC8()); // decoder.cpp:85 (never freed there either)
    return dec;
}

Decoder* create(size_t blockLength, size_t listSize, const std::vector<unsigned>& frozenBits, std::string type)
{
    std::transform(type.begin(), type.end(), type.begin(), [](unsigned char c) { return std::tolower(c); });
    // decoder.cpp:35-51: "char" is tested first, then "float", "mixed", "scan"; list size < 2
    // turns every non-char type into the float Fast-SSC decoder
    int flag;
    if (type.find("char") != std::string::npos)
        flag = 0;
    else if (type.find("gpu") != std::string::npos || type.find("float") != std::string::npos)
        flag = 1;
    else if (type.find("mixed") != std::string::npos)
        flag = 2;
    else if (type.find("scan") != std::string::npos)
        flag = 3;
    else
        throw std::logic_error("Unknown PolarDecoder type!");
    if (listSize < 2 && flag != 0)
        flag = 1;
    return makeDecoder(blockLength, listSize, frozenBits, flag);
}

} // namespace Decoding
} // namespace PolarCode
