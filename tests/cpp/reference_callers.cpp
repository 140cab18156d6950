// The reference's own callers, written against this build's headers exactly as they are in
// the reference (include paths, class names, call sequences), compiled with g++ and linked
// with libpolarcode_amd.so (tests/test_cpp_boundary.py builds and runs it).
//
//   encode <N> <sys> <crc> <frozen.txt> <info.bin>   the simulator's encoder sequence
//        (src/simulation/simulator.cpp:703-705, 843-847, 869-875): ButterflyFipPacked,
//        setInformation -> encode -> getEncodedData into a PackedContainer; prints the code
//        bytes (hex) and the check-bit-filled information bytes
//   api                                              CPU-only contract checks (below)
//   gpu <frozen.txt> <llr.bin> <F>                   the simulator's decoder sequence
//        (simulator.cpp:703-764, 920-937) on the GPU: setCoders' decoder classes by their
//        reference names, setSignal -> decode -> packedOutput; prints one line per frame
#include <polarcode/bitcontainer.h>
#include <polarcode/construction/bhattacharrya.h>
#include <polarcode/decoding/adaptive_char.h>
#include <polarcode/decoding/adaptive_float.h>
#include <polarcode/decoding/adaptive_mixed.h>
#include <polarcode/decoding/decoder.h>
#include <polarcode/decoding/fastssc_avx_float.h>
#include <polarcode/decoding/fastssc_fip_char.h>
#include <polarcode/decoding/scl_avx_float.h>
#include <polarcode/decoding/scl_fip_char.h>
#include <polarcode/encoding/butterfly_fip_packed.h>
#include <polarcode/encoding/encoder.h>
#include <polarcode/errordetection/crc32.h>
#include <polarcode/errordetection/crc8.h>
#include <polarcode/errordetection/dummy.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

using namespace PolarCode;

#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "FAILED: %s (line %d)\n", #c, __LINE__);                        \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

static std::vector<unsigned> read_frozen(const char* path)
{
    std::vector<unsigned> f;
    std::ifstream in(path);
    unsigned v;
    while (in >> v)
        f.push_back(v);
    return f;
}

static std::vector<char> read_bytes(const char* path)
{
    std::ifstream in(path, std::ios::binary);
    return std::vector<char>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

static void hex(const unsigned char* p, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        std::printf("%02x", p[i]);
}

// A reference-style Encoder subclass: overrides encode() only and works on the base's
// protected state (xmInputData, mBitContainer, mCodewordReady, mErrorDetector, mFrozenBits),
// like the reference's RecursiveFipPacked.  Its transform is the naive O(N^2) G_N product.
class MatrixEncoder : public Encoding::Encoder
{
public:
    MatrixEncoder(size_t N, const std::vector<unsigned>& frozen) { initialize(N, frozen); }
    void initialize(size_t N, const std::vector<unsigned>& frozen) override
    {
        mBlockLength = N;
        mFrozenBits = frozen;
        delete mBitContainer;
        mBitContainer = new PackedContainer(N, mFrozenBits);
    }
    void encode() override
    {
        if (!mCodewordReady) {
            mErrorDetector->generate(xmInputData, (int)(infoLength() / 8));
            mBitContainer->insertPackedInformationBits(xmInputData);
        }
        matrix();
        if (mSystematic) {
            clearFrozenBits();
            matrix();
        }
        mCodewordReady = false;
    }

private:
    void matrix()
    {
        const size_t N = mBlockLength;
        std::vector<unsigned char> u(N / 8), x(N / 8, 0);
        mBitContainer->getPackedBits(u.data());
        // x = u G_N without bit reversal (the reference's x[i] ^= x[i + 2^s] butterflies):
        // x_j = XOR of u_i over every i whose bits include j's
        for (size_t j = 0; j < N; ++j) {
            unsigned b = 0;
            for (size_t i = 0; i < N; ++i)
                if ((i & j) == j)
                    b ^= (u[i / 8] >> (7 - i % 8)) & 1u;
            x[j / 8] |= (unsigned char)(b << (7 - j % 8));
        }
        mBitContainer->insertPackedBits(x.data());
    }
};

static int run_encode(int argc, char** argv)
{
    CHECK(argc == 7);
    const size_t N = std::strtoul(argv[2], nullptr, 10);
    const bool sys = std::atoi(argv[3]) != 0;
    const int crc = std::atoi(argv[4]);
    std::vector<unsigned> frozen = read_frozen(argv[5]);
    std::vector<char> info = read_bytes(argv[6]);
    const size_t K = N - frozen.size(), kb = (K + 7) / 8; // the simulator uses K / 8 (K % 8 == 0)
    CHECK(info.size() >= kb);
    ErrorDetection::Detector* det = ErrorDetection::create((unsigned)crc, "crc");
    // simulator.cpp:703-705 (setCoders), 843-847 (buffers), 869-875 (encode)
    Encoding::Encoder* mEncoder = new Encoding::ButterflyFipPacked(N, frozen);
    mEncoder->setSystematic(sys);
    mEncoder->setErrorDetection(det);
    unsigned char* mInputData = new unsigned char[kb];
    std::memcpy(mInputData, info.data(), kb);
    PackedContainer* mEncodedData = new PackedContainer(N);
    mEncoder->setInformation(mInputData);
    mEncoder->encode();
    mEncoder->getEncodedData(mEncodedData->data());
    // the same through encode_vector and through the reference-style subclass
    std::vector<unsigned char> again(info.begin(), info.begin() + kb), code2(N / 8), code3(N / 8);
    std::vector<unsigned char> again3 = again;
    mEncoder->encode_vector(again.data(), code2.data());
    MatrixEncoder me(N, frozen);
    me.setSystematic(sys);
    me.setErrorDetection(det);
    me.encode_vector(again3.data(), code3.data());
    // read back as the simulator's modulator does (Modem::setInputData -> getFloatBits,
    // modem.cpp:29-37); getEncodedData wrote at the buffer's start and getFloatBits reads
    // from there for every N, as in the reference
    std::vector<float> fb(N);
    mEncodedData->getFloatBits(fb.data());
    std::vector<unsigned char> code(N / 8, 0);
    for (size_t i = 0; i < N; ++i)
        code[i / 8] |= (unsigned char)((std::signbit(fb[i]) ? 1u : 0u) << (7 - i % 8));
    CHECK(std::memcmp(code.data(), code2.data(), N / 8) == 0);
    CHECK(std::memcmp(code.data(), code3.data(), N / 8) == 0);
    CHECK(std::memcmp(mInputData, again.data(), kb) == 0 && std::memcmp(mInputData, again3.data(), kb) == 0);
    // systematic: the information bits are readable from the codeword (getInformation)
    if (sys) {
        std::vector<unsigned char> back(kb);
        mEncoder->getInformation(back.data());
        for (size_t j = 0; j < K; ++j)
            CHECK(((back[j / 8] ^ mInputData[j / 8]) >> (7 - j % 8) & 1u) == 0);
    }
    hex(code.data(), N / 8);
    std::printf(" ");
    hex(mInputData, kb);
    std::printf("\n");
    delete mEncodedData;
    delete[] mInputData;
    delete mEncoder;
    delete det;
    return 0;
}

static int run_api()
{
    const std::vector<unsigned> fr = Construction::frozen_bits(1024, 512, 0.0f, "BB");
    // makeDecoder(N, L, frozen) without an implementation builds the 8-bit decoders
    // (decoder.h:196-199 default 0; decoder.cpp:60-83), with CRC-8 installed (Q5)
    {
        std::unique_ptr<Decoding::Decoder> d(Decoding::makeDecoder(1024, 8, fr));
        CHECK(dynamic_cast<Decoding::SclFipChar*>(d.get()) != nullptr);
        CHECK(d->getErrorDetectionMode() == "CRC-8" && d->getListSize() == 8);
        CHECK(dynamic_cast<CharContainer*>(d->inputContainer()) != nullptr);
        CHECK(dynamic_cast<CharContainer*>(d->outputContainer()) != nullptr);
        std::unique_ptr<Decoding::Decoder> s(Decoding::makeDecoder(1024, 1, fr));
        CHECK(dynamic_cast<Decoding::FastSscFipChar*>(s.get()) != nullptr);
        // unknown implementations take the 8-bit default branch as well
        std::unique_ptr<Decoding::Decoder> u(Decoding::makeDecoder(1024, 4, fr, 7));
        CHECK(dynamic_cast<Decoding::SclFipChar*>(u.get()) != nullptr);
        std::unique_ptr<Decoding::Decoder> f(Decoding::makeDecoder(1024, 4, fr, 1));
        CHECK(dynamic_cast<Decoding::SclAvxFloat*>(f.get()) != nullptr);
        CHECK(dynamic_cast<FloatContainer*>(f->inputContainer()) != nullptr);
        std::unique_ptr<Decoding::Decoder> a(Decoding::makeDecoder(1024, 4, fr, 2));
        CHECK(dynamic_cast<Decoding::AdaptiveFloat*>(a.get()) != nullptr);
        CHECK(a->getErrorDetectionMode() == "DUMMY-0"); // AdaptiveFloat passes detectors to its stages
        bool threw = false;
        try {
            delete Decoding::makeDecoder(1024, 4, fr, 3);
        } catch (const std::logic_error&) {
            threw = true; // SCAN is outside this build
        }
        CHECK(threw);
    }
    // setCoders' classes construct by their reference names without a GPU
    std::unique_ptr<Decoding::Decoder> d1(new Decoding::FastSscAvxFloat(1024, fr));
    std::unique_ptr<Decoding::Decoder> d2(new Decoding::AdaptiveFloat(1024, 8, fr));
    std::unique_ptr<Decoding::Decoder> d3(new Decoding::AdaptiveMixed(1024, 8, fr));
    std::unique_ptr<Decoding::Decoder> d4(new Decoding::AdaptiveChar(1024, 8, fr));
    std::unique_ptr<Decoding::Decoder> d5(new Decoding::FastSscFipChar(1024, fr));
    CHECK(d3->getListSize() == 8 && d3->inputContainer() == nullptr);
    // BitContainer round trips in the reference's formats
    {
        std::vector<unsigned> f8 = { 0, 1, 2, 4 };
        FloatContainer fc(8, f8);
        unsigned char info = 0xA0; // 4 info bits: 1010
        fc.insertPackedInformationBits(&info);
        unsigned char back = 0;
        fc.getPackedInformationBits(&back);
        CHECK(back == 0xA0);
        float fb[8];
        fc.getFloatBits(fb);
        CHECK(std::signbit(fb[3]) && !std::signbit(fb[5]) && std::signbit(fb[6]) && !std::signbit(fb[7]));
        CharContainer cc(32);
        std::vector<float> x(32, 0.5f);
        x[1] = 1.5f;   // nearest even -> 2
        x[2] = -200.f; // saturates
        x[3] = NAN;    // cvtps_epi32 -> INT_MIN -> -128
        x[4] = 3e9f;   // out of range -> INT_MIN -> -128
        cc.insertLlr(x.data());
        CHECK(cc.data()[0] == 0 && cc.data()[1] == 2 && cc.data()[2] == -128 && cc.data()[3] == -128 &&
              cc.data()[4] == -128);
        PackedContainer pc(16, f8);
        unsigned char code[2] = { 0xFF, 0xFF };
        pc.insertPackedBits(code);
        pc.resetFrozenBits();
        pc.getPackedBits(code);
        CHECK(code[0] == 0x17 /* 0,1,2,4 cleared */ && code[1] == 0xFF);
    }
    std::printf("api ok\n");
    return 0;
}

static void packed_signs(BitContainer* c, size_t N, unsigned char* out)
{
    std::vector<float> fb(N);
    c->getFloatBits(fb.data());
    std::memset(out, 0, N / 8);
    for (size_t i = 0; i < N; ++i)
        out[i / 8] |= (unsigned char)((std::signbit(fb[i]) ? 1u : 0u) << (7 - i % 8));
}

static int run_gpu(int argc, char** argv)
{
    CHECK(argc == 5);
    std::vector<unsigned> frozen = read_frozen(argv[2]);
    std::vector<char> raw = read_bytes(argv[3]);
    const size_t F = std::strtoul(argv[4], nullptr, 10), N = 1024;
    CHECK(raw.size() == F * N * sizeof(float));
    const float* llr = reinterpret_cast<const float*>(raw.data());
    ErrorDetection::CRC8 crc;
    // setCoders (simulator.cpp:721-758): precision 32 L=1 / L=8, precision 832 L=8
    std::vector<std::unique_ptr<Decoding::Decoder>> decs;
    decs.emplace_back(new Decoding::FastSscAvxFloat(N, frozen));
    decs.emplace_back(new Decoding::AdaptiveFloat(N, 8, frozen));
    decs.emplace_back(new Decoding::AdaptiveMixed(N, 8, frozen));
    decs.emplace_back(new Decoding::SclAvxFloat(N, 8, frozen));
    for (auto& d : decs) {
        d->setSystematic(true);
        d->setErrorDetection(&crc);
    }
    for (size_t k = 0; k < decs.size(); ++k) {
        Decoding::Decoder* mDecoder = decs[k].get();
        for (size_t f = 0; f < F; ++f) {
            // simulator.cpp:920-937
            mDecoder->setSignal(llr + f * N);
            const bool success = mDecoder->decode();
            unsigned char* mDecodedData = mDecoder->packedOutput();
            std::printf("%zu %zu %d ", k, f, success ? 1 : 0);
            hex(mDecodedData, (N - frozen.size()) / 8);
            // the output container holds the decoded codeword (its sign bits: getFloatBits; the
            // reference's getPackedBits is exact for +-0.0 "bits" only, not for a soft codeword)
            std::vector<unsigned char> cw(N / 8);
            packed_signs(mDecoder->outputContainer(), N, cw.data());
            std::printf(" ");
            hex(cw.data(), N / 8);
            // getSoftCodeword (decoder.cpp:147): the reference's soft codeword (Fast-SSC float) or
            // the selected path's signed hard decisions (list / adaptive decoders); its signs
            // (AdaptiveMixed's container is its 8-bit stage's CharContainer when that stage succeeded,
            // as in the reference: char bits then)
            const bool chars = dynamic_cast<CharContainer*>(mDecoder->outputContainer()) != nullptr;
            std::vector<float> sw(N);
            mDecoder->getSoftCodeword(sw.data());
            const signed char* sb = reinterpret_cast<const signed char*>(sw.data());
            std::vector<unsigned char> sc(N / 8, 0);
            for (size_t i = 0; i < N; ++i)
                sc[i / 8] |= (unsigned char)(((chars ? sb[i] < 0 : std::signbit(sw[i])) ? 1u : 0u) << (7 - i % 8));
            std::printf(" ");
            hex(sc.data(), N / 8);
            std::printf("\n");
        }
    }
    // Fast-SSC float: the soft codeword of the last frame, its signs = the codeword bits
    std::vector<float> soft(N);
    decs[0]->setSignal(llr);
    decs[0]->decode();
    decs[0]->getSoftCodeword(soft.data());
    std::vector<unsigned char> cw(N / 8);
    packed_signs(decs[0]->outputContainer(), N, cw.data());
    for (size_t i = 0; i < N; ++i)
        CHECK(((cw[i / 8] >> (7 - i % 8)) & 1u) == (std::signbit(soft[i]) ? 1u : 0u));
    // SclAvxFloat: getSoftInformation = the soft codeword at the information positions
    std::vector<float> si(N - frozen.size());
    decs[3]->setSignal(llr);
    decs[3]->decode();
    decs[3]->getSoftCodeword(soft.data());
    decs[3]->getSoftInformation(si.data());
    std::vector<char> isfz(N, 0);
    for (unsigned f : frozen)
        isfz[f] = 1;
    for (size_t i = 0, j = 0; i < N; ++i)
        if (!isfz[i])
            CHECK(std::memcmp(&soft[i], &si[j++], sizeof(float)) == 0);
    std::printf("gpu ok\n");
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 2)
        return 2;
    const std::string mode = argv[1];
    if (mode == "encode")
        return run_encode(argc, argv);
    if (mode == "api")
        return run_api();
    if (mode == "gpu")
        return run_gpu(argc, argv);
    return 2;
}
