// A Decoder subclass written the way the reference's own decoders are (containers created in
// initialize(), decode() reads mLlrContainer and fills mOutputContainer, the base's
// setSignal / decode_vector / getDecodedInformationBits / destructor do the rest), compiled
// against this build's include/polarcode/decoding/decoder.h and linked with
// libpolarcode_amd.so.  Checks that the base class keeps the reference's contract: the
// batch methods have working defaults, setSignal(const char*) converts bytes for float
// containers, the containers are BitContainers, and the GPU factory validates codes without a
// GPU.  (tests/test_cpp_boundary.py builds and runs it.)
#include <polarcode/bitcontainer.h>
#include <polarcode/decoding/decoder.h>
#include <polarcode/errordetection/errordetector.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

using namespace PolarCode;

// "Repeat the sign of LLR 0 into every info bit" -- a toy decoder, like a user's own subclass
class SignDecoder : public Decoding::Decoder
{
public:
    SignDecoder(size_t n, const std::vector<unsigned>& frozen) { initialize(n, frozen); }
    void initialize(size_t n, const std::vector<unsigned>& frozen) override
    {
        Decoder::initialize(n, frozen);
        mLlrContainer = new FloatContainer(n);
        mBitContainer = new FloatContainer(n, frozen);
        mOutputContainer = new unsigned char[(n - frozen.size() + 7) / 8];
    }
    bool decode() override
    {
        const float* llr = static_cast<FloatContainer*>(mLlrContainer)->data();
        const unsigned char b = llr[0] < 0.0f ? 0xff : 0x00;
        std::memset(mOutputContainer, b, infoLength() / 8);
        mBitContainer->insertPackedInformationBits(mOutputContainer);
        return llr[0] != 0.0f;
    }
};

#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (!(c)) {                                                                               \
            std::fprintf(stderr, "FAILED: %s (line %d)\n", #c, __LINE__);                        \
            return 1;                                                                             \
        }                                                                                         \
    } while (0)

int main()
{
    std::vector<unsigned> frozen;
    for (unsigned i = 0; i < 8; ++i)
        frozen.push_back(i);
    SignDecoder d(16, frozen);
    CHECK(d.blockLength() == 16 && d.infoLength() == 8 && d.getListSize() == 1);
    // decode_vector and the default decodeBatch (a decode_vector loop) agree
    std::vector<float> llr(3 * 16, 1.0f);
    llr[16] = -2.0f; // frame 1 negative
    llr[32] = 0.0f;  // frame 2 "fails"
    unsigned char one = 0;
    CHECK(d.decode_vector(llr.data() + 16, &one) && one == 0xff && d.packedOutput()[0] == 0xff);
    std::vector<uint8_t> info(3), ok(3);
    CHECK(!d.decodeBatch(llr.data(), 3, info.data(), ok.data()));
    CHECK(info[0] == 0x00 && info[1] == 0xff && ok[0] == 1 && ok[1] == 1 && ok[2] == 0);
    // setSignal(const char*) is the base's non-virtual conversion through the FloatContainer
    std::vector<char> c8(16, 5);
    c8[0] = -3;
    CHECK(d.decode_vector(c8.data(), &one) && one == 0xff);
    std::vector<float> frame(16);
    d.inputContainer()->getSoftBits(frame.data());
    CHECK(frame[0] == -3.0f && frame[1] == 5.0f);
    std::vector<int8_t> b8(2 * 16, 1);
    CHECK(d.decodeBatchI8(b8.data(), 2, info.data(), ok.data()) && info[0] == 0);
    // the output container is a BitContainer: packed bits / soft information as the reference
    d.decode_vector(llr.data() + 16, &one);
    unsigned char packed[2] = { 0, 0 };
    d.outputContainer()->getPackedBits(packed);
    CHECK(packed[0] == 0x00 && packed[1] == 0xff);
    std::vector<float> si(8);
    d.getSoftInformation(si.data());
    CHECK(std::signbit(si[0]) && std::signbit(si[7]));
    // the device batch is not available on a CPU decoder: loud failure
    bool threw = false;
    try {
        d.decodeBatchDevice(nullptr, 1, nullptr);
    } catch (const std::logic_error&) {
        threw = true;
    }
    CHECK(threw);
    // the GPU factory classifies (and rejects) codes like the reference without a GPU
    threw = false;
    try {
        std::vector<unsigned> bad = { 1, 2 }; // DoubleRep pattern not starting at 0 (invalid_argument)
        delete Decoding::create(4, 1, bad, "gpu");
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    CHECK(threw);
    threw = false;
    try {
        delete Decoding::create(16, 1, frozen, "no such type");
    } catch (const std::logic_error& e) {
        threw = std::strcmp(e.what(), "Unknown PolarDecoder type!") == 0;
    }
    CHECK(threw);
    std::printf("subclass_decoder ok\n");
    return 0;
}
