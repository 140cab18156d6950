/* -*- c++ -*- */
// <polarcode/decoding/adaptive_mixed.h> of the reference: `AdaptiveMixed` (src/polarcode/decoding/adaptive_mixed.cpp) is this build's GPU
// decoder GpuAdaptiveMixed (include/polarcode/decoding/decoder.h) -- same constructor (N, listSize, frozenBits),
// same Decoder interface -- so callers such as the reference simulator's setCoders
// (src/simulation/simulator.cpp:703-764) compile unchanged and decode on the MI355X.
#ifndef PCA_DECODING_ADAPTIVE_MIXED_H
#define PCA_DECODING_ADAPTIVE_MIXED_H

#include <polarcode/decoding/decoder.h>

namespace PolarCode {
namespace Decoding {

using AdaptiveMixed = GpuAdaptiveMixed;

} // namespace Decoding
} // namespace PolarCode

#endif
