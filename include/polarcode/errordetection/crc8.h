/* -*- c++ -*- */
// <polarcode/errordetection/crc8.h> of the reference: CRC8 (crc8.cpp) is declared in
// <polarcode/errordetection/errordetector.h> in this build; this header keeps the reference's include path.
#ifndef PCA_ERRORDETECTION_CRC8_H
#define PCA_ERRORDETECTION_CRC8_H

#include <polarcode/errordetection/errordetector.h>

#endif
