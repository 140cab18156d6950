/* -*- c++ -*- */
// <polarcode/construction/bhattacharrya.h> of the reference: Bhattacharrya (bhattacharrya.cpp) is declared in
// <polarcode/construction/constructor.h> in this build; this header keeps the reference's include path.
#ifndef PCA_CONSTRUCTION_BHATTACHARRYA_H
#define PCA_CONSTRUCTION_BHATTACHARRYA_H

#include <polarcode/construction/constructor.h>

#endif
