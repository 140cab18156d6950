#!/bin/bash
# round 4, first call: the GPU suite (specialised kernels at every config), the staging-layout
# A/B on SCL-8 and the LDS bank-conflict counters of both layouts
set -o pipefail
T=r04a
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/$T/gputest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/gputest.log | head -20; exit 1; }
timeout -k 10 900 bash tools/sweep_libs.sh scl8 $T/ab "-|PCG_NONE=1" "stg0|PCG_NONE=1" "-|PCG_RTC_SCL=0" "stg0|PCG_RTC_SCL=0" || exit 1
timeout -k 10 400 bash tools/pmc_scl8.sh scl8 $T/pmc_gm1 || exit 1
timeout -k 10 400 bash tools/pmc_scl8.sh scl8 $T/pmc_gm0 PCG_DEV_LIB=lib_dev/libpcg_stg0.so || exit 1
