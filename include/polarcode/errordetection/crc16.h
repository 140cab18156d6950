/* -*- c++ -*- */
// <polarcode/errordetection/crc16.h> of the reference: CRC16 (crc16.cpp) is declared in
// <polarcode/errordetection/errordetector.h> in this build; this header keeps the reference's include path.
#ifndef PCA_ERRORDETECTION_CRC16_H
#define PCA_ERRORDETECTION_CRC16_H

#include <polarcode/errordetection/errordetector.h>

#endif
