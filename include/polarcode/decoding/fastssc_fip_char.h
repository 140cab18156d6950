/* -*- c++ -*- */
// <polarcode/decoding/fastssc_fip_char.h> of the reference: `FastSscFipChar` (src/polarcode/decoding/fastssc_fip_char.cpp) is this build's GPU
// decoder GpuFastSscChar (include/polarcode/decoding/decoder.h) -- same constructor (N, frozenBits),
// same Decoder interface -- so callers such as the reference simulator's setCoders
// (src/simulation/simulator.cpp:703-764) compile unchanged and decode on the MI355X.
#ifndef PCA_DECODING_FASTSSC_FIP_CHAR_H
#define PCA_DECODING_FASTSSC_FIP_CHAR_H

#include <polarcode/decoding/decoder.h>

namespace PolarCode {
namespace Decoding {

using FastSscFipChar = GpuFastSscChar;

} // namespace Decoding
} // namespace PolarCode

#endif
