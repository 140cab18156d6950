/* -*- c++ -*- */
// <polarcode/decoding/adaptive_char.h> of the reference: `AdaptiveChar` (src/polarcode/decoding/adaptive_char.cpp) is this build's GPU
// decoder GpuAdaptiveChar (include/polarcode/decoding/decoder.h) -- same constructor (N, listSize, frozenBits),
// same Decoder interface -- so callers such as the reference simulator's setCoders
// (src/simulation/simulator.cpp:703-764) compile unchanged and decode on the MI355X.
#ifndef PCA_DECODING_ADAPTIVE_CHAR_H
#define PCA_DECODING_ADAPTIVE_CHAR_H

#include <polarcode/decoding/decoder.h>

namespace PolarCode {
namespace Decoding {

using AdaptiveChar = GpuAdaptiveChar;

} // namespace Decoding
} // namespace PolarCode

#endif
