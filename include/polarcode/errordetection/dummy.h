/* -*- c++ -*- */
// <polarcode/errordetection/dummy.h> of the reference: Dummy and globalDummyDetector (dummy.cpp) is declared in
// <polarcode/errordetection/errordetector.h> in this build; this header keeps the reference's include path.
#ifndef PCA_ERRORDETECTION_DUMMY_H
#define PCA_ERRORDETECTION_DUMMY_H

#include <polarcode/errordetection/errordetector.h>

#endif
