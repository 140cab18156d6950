/* -*- c++ -*- */
// PolarCode::Construction -- frozen-set construction (host side), the reference's
// interface (include/polarcode/construction/constructor.h:20-62,
// bhattacharrya.h, fiveGList.h in david13pod/antPolarCodes).
#ifndef PCA_CONSTRUCTOR_H
#define PCA_CONSTRUCTOR_H

#include <cstddef>
#include <string>
#include <vector>

namespace PolarCode {
namespace Construction {

/// Constructor base (constructor.h:20-57): lengths + design SNR, construct() = frozen set
/// (ascending).  setBlockLength throws std::invalid_argument("new blockLength is not a
/// power of 2!") like constructor.cpp:25-32.
class Constructor
{
protected:
    size_t mBlockLength = 0;
    size_t mInformationLength = 0;
    float mDesignSnr = 0.0f;

public:
    Constructor() {}
    virtual ~Constructor() {}
    virtual std::vector<unsigned> construct() = 0;
    void setBlockLength(size_t newBlockLength);
    void setInformationLength(size_t newInformationLength) { mInformationLength = newInformationLength; }
    void setDesignSnr(float designSnr) { mDesignSnr = designSnr; }
};

/// Bhattacharyya bounds (bhattacharrya.cpp:39-82): float initial parameter, double
/// recursion, stable descending sort, the N-K least reliable sub-channels frozen.
class Bhattacharrya : public Constructor
{
public:
    Bhattacharrya() {}
    Bhattacharrya(size_t N, size_t K, float designSnr = 0.0f);
    std::vector<unsigned> construct() override;
};

/// 3GPP TS 38.212 reliability sequence (fiveGList.cpp:19-37): N > 1024 throws
/// std::invalid_argument; K > N throws std::invalid_argument("Invalid polar code(N, K)");
/// the first N-K entries of the N = 1024 sequence are frozen for every N.
class FiveGList : public Constructor
{
public:
    FiveGList() {}
    FiveGList(size_t N, size_t K);
    FiveGList(size_t N, size_t K, float /*designSnr, unused*/) : FiveGList(N, K) {}
    std::vector<unsigned> construct() override;
};

/// Beta expansion (betaexpansion.cpp:39-78): weight(i) = sum_j bit_j(i) * 2^(j/4), the N-K
/// lightest sub-channels frozen (std::sort order, ties as libstdc++ leaves them).
class BetaExpansion : public Constructor
{
public:
    BetaExpansion() {}
    BetaExpansion(size_t N, size_t K);
    BetaExpansion(size_t N, size_t K, float /*designSnr, unused*/) : BetaExpansion(N, K) {}
    std::vector<unsigned> construct() override;
};

/// Construction::frozen_bits (constructor.cpp:41-63): type matched case-insensitively by
/// substring, "be" -> BetaExpansion, "5g" -> FiveGList, anything else -> Bhattacharrya
/// ("BB", the default).
std::vector<unsigned> frozen_bits(const int blockLength,
                                  const int infoLength,
                                  const float designSNR,
                                  const std::string& constructor_type = std::string("BB"));

} // namespace Construction
} // namespace PolarCode

#endif
