/* -*- c++ -*- */
// <polarcode/decoding/adaptive_float.h> of the reference: `AdaptiveFloat` (src/polarcode/decoding/adaptive_float.cpp) is this build's GPU
// decoder GpuAdaptiveFloat (include/polarcode/decoding/decoder.h) -- same constructor (N, listSize, frozenBits),
// same Decoder interface -- so callers such as the reference simulator's setCoders
// (src/simulation/simulator.cpp:703-764) compile unchanged and decode on the MI355X.
#ifndef PCA_DECODING_ADAPTIVE_FLOAT_H
#define PCA_DECODING_ADAPTIVE_FLOAT_H

#include <polarcode/decoding/decoder.h>

namespace PolarCode {
namespace Decoding {

using AdaptiveFloat = GpuAdaptiveFloat;

} // namespace Decoding
} // namespace PolarCode

#endif
