#!/bin/bash
# SCL-8 at three waves per SIMD: the list kernel bounded to 168 VGPRs (PCG_LS_MINW=3, 58
# spilled statically) with 13 / 12 KB LDS per wave (12 waves per CU) against HEAD (2 waves per
# SIMD, 20 KB); code objects pre-compiled into lib_dev/rtc
set -o pipefail
T=r04n
mkdir -p gpurun_out/$T
C=PCG_RTC_CACHE=lib_dev/rtc
timeout -k 10 900 bash tools/sweep_libs.sh scl8 $T/minw3 "-|PCG_NONE=1" "minw3_8|$C PCG_SCL_LDS_KB=13" "minw3_8|$C PCG_SCL_LDS_KB=12" || exit 1
