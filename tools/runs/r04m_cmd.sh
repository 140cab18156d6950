#!/bin/bash
# config 5: the recomputed eighths (virt 3, the default at LP >= 16) against virt 2 on the
# specialised kernel (static: 49 vs 25 spilled VGPRs), code objects pre-compiled into lib_dev/rtc
set -o pipefail
T=r04m
mkdir -p gpurun_out/$T
C=PCG_RTC_CACHE=lib_dev/rtc
timeout -k 10 900 bash tools/sweep_libs.sh scl32 $T/virt "-|PCG_NONE=1" "-|$C PCG_SCL_VIRT=2" "-|$C PCG_SCL_VIRT=2 PCG_SCL_V3=2" || exit 1
