/* -*- c++ -*- */
// <polarcode/errordetection/crc32.h> of the reference: CRC32 (crc32.cpp, CRC-32C) is declared in
// <polarcode/errordetection/errordetector.h> in this build; this header keeps the reference's include path.
#ifndef PCA_ERRORDETECTION_CRC32_H
#define PCA_ERRORDETECTION_CRC32_H

#include <polarcode/errordetection/errordetector.h>

#endif
