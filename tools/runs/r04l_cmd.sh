#!/bin/bash
# SCL-8 (config 3) under four machine-scheduler strategies for the specialised kernel
# (PCG_RTC_XOPTS; code objects pre-compiled into lib_dev/rtc by tools/warm_dev.py)
set -o pipefail
T=r04l
mkdir -p gpurun_out/$T
C=PCG_RTC_CACHE=lib_dev/rtc
timeout -k 10 900 bash tools/sweep_libs.sh scl8 $T/sched "-|PCG_NONE=1" \
    "-|$C PCG_RTC_XOPTS=-mllvm,-amdgpu-sched-strategy=max-ilp" \
    "-|$C PCG_RTC_XOPTS=-mllvm,-amdgpu-schedule-metric-bias=0" \
    "-|$C PCG_RTC_XOPTS=-mllvm,-amdgpu-use-amdgpu-trackers" \
    "-|$C PCG_RTC_XOPTS=-mllvm,-amdgpu-sched-strategy=max-memory-clause" || exit 1
