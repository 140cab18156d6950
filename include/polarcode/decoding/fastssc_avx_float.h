/* -*- c++ -*- */
// <polarcode/decoding/fastssc_avx_float.h> of the reference: `FastSscAvxFloat` (src/polarcode/decoding/fastssc_avx_float.cpp) is this build's GPU
// decoder GpuFastSscFloat (include/polarcode/decoding/decoder.h) -- same constructor (N, frozenBits),
// same Decoder interface -- so callers such as the reference simulator's setCoders
// (src/simulation/simulator.cpp:703-764) compile unchanged and decode on the MI355X.
#ifndef PCA_DECODING_FASTSSC_AVX_FLOAT_H
#define PCA_DECODING_FASTSSC_AVX_FLOAT_H

#include <polarcode/decoding/decoder.h>

namespace PolarCode {
namespace Decoding {

using FastSscAvxFloat = GpuFastSscFloat;

} // namespace Decoding
} // namespace PolarCode

#endif
