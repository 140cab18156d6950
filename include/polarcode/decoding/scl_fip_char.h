/* -*- c++ -*- */
// <polarcode/decoding/scl_fip_char.h> of the reference: `SclFipChar` (src/polarcode/decoding/scl_fip_char.cpp) is this build's GPU
// decoder GpuSclChar (include/polarcode/decoding/decoder.h) -- same constructor (N, listSize, frozenBits),
// same Decoder interface -- so callers such as the reference simulator's setCoders
// (src/simulation/simulator.cpp:703-764) compile unchanged and decode on the MI355X.
#ifndef PCA_DECODING_SCL_FIP_CHAR_H
#define PCA_DECODING_SCL_FIP_CHAR_H

#include <polarcode/decoding/decoder.h>

namespace PolarCode {
namespace Decoding {

using SclFipChar = GpuSclChar;

} // namespace Decoding
} // namespace PolarCode

#endif
