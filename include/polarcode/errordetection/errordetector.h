/* -*- c++ -*- */
// PolarCode::ErrorDetection -- the reference's detector interface
// (include/polarcode/errordetection/errordetector.h:24-81 in david13pod/antPolarCodes),
// host-side.  The GPU decoders read getType()/getCheckBitCount() to pick the
// device-side syndrome (pcg.h PCG_CRC*); CMAC is not part of this build.
#ifndef PCA_ERRORDETECTOR_H
#define PCA_ERRORDETECTOR_H

#include <string>

namespace PolarCode {
namespace ErrorDetection {

class Detector
{
public:
    Detector() {}
    virtual ~Detector() {}
    virtual unsigned getCheckBitCount() = 0;
    virtual std::string getType() = 0;
    virtual void generate(void* data, int bytes) = 0;
    virtual bool check(void* data, int bytes) = 0;
    virtual int multiCheck(void** data, int nArrays, int nBytes) = 0;
};

/// Dummy (dummy.cpp:14-31): check() always true.
class Dummy : public Detector
{
public:
    unsigned getCheckBitCount() override { return 0; }
    std::string getType() override { return "DUMMY"; }
    void generate(void*, int) override {}
    bool check(void*, int) override { return true; }
    int multiCheck(void**, int, int) override { return 0; }
};

/// CRC-8 poly 0x07, CRC-16/CCITT-FALSE, CRC-32C (crc8.cpp, crc16.cpp, crc32.cpp)
class Crc : public Detector
{
    unsigned mBits;

public:
    explicit Crc(unsigned bits) : mBits(bits) {}
    unsigned getCheckBitCount() override { return mBits; }
    std::string getType() override { return "CRC"; }
    void generate(void* data, int bytes) override;
    bool check(void* data, int bytes) override;
    int multiCheck(void** data, int nArrays, int nBytes) override;
};

class CRC8 : public Crc
{
public:
    CRC8() : Crc(8) {}
};
/// 3GPP TS 38.212 CRC-11 (gCRC11 = D^11+D^10+D^9+D^5+1, zero init) over the message bit
/// stream, parity in the last 11 bits.  NOT in the reference: added for the
/// 5G NR uplink chain (config 4); ErrorDetection::create(11, "crc") returns it.
class CRC11 : public Crc
{
public:
    CRC11() : Crc(11) {}
};
class CRC16 : public Crc
{
public:
    CRC16() : Crc(16) {}
};
class CRC32 : public Crc
{
public:
    CRC32() : Crc(32) {}
};

extern Dummy globalDummyDetector;

/// ErrorDetection::create (errordetector.cpp:23-67): "crc" sizes 0/8/16/32, plus 11 (CRC11,
/// this build's extension) (std::logic_error("CRC INVALID SIZE!") otherwise); "cmac" -> std::logic_error (not
/// in this build); anything else std::runtime_error("Unknown Error detector requested!").
Detector* create(unsigned size, std::string type);

/// pcg.h crc kind for a detector (0, 8, 11, 16, 32); -1 if the GPU cannot evaluate it.
int gpuKind(Detector* d);

} // namespace ErrorDetection
} // namespace PolarCode

#endif
