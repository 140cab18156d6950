/* -*- c++ -*- */
// <polarcode/construction/betaexpansion.h> of the reference: BetaExpansion (betaexpansion.cpp) is declared in
// <polarcode/construction/constructor.h> in this build; this header keeps the reference's include path.
#ifndef PCA_CONSTRUCTION_BETAEXPANSION_H
#define PCA_CONSTRUCTION_BETAEXPANSION_H

#include <polarcode/construction/constructor.h>

#endif
