/* -*- c++ -*- */
// PolarCode::Construction::frozen_bits (constructor.h:58-62 of the reference).
#ifndef PCA_CONSTRUCTOR_H
#define PCA_CONSTRUCTOR_H

#include <string>
#include <vector>

namespace PolarCode {
namespace Construction {

/// "BB" (Bhattacharyya bounds, bhattacharrya.cpp:39-82) -- the reference default.
std::vector<unsigned> frozen_bits(const int blockLength,
                                  const int infoLength,
                                  const float designSNR,
                                  const std::string& constructor_type = std::string("BB"));

} // namespace Construction
} // namespace PolarCode

#endif
