/* -*- c++ -*- */
// <polarcode/construction/fiveGList.h> of the reference: FiveGList (fiveGList.cpp) is declared in
// <polarcode/construction/constructor.h> in this build; this header keeps the reference's include path.
#ifndef PCA_CONSTRUCTION_FIVEGLIST_H
#define PCA_CONSTRUCTION_FIVEGLIST_H

#include <polarcode/construction/constructor.h>

#endif
