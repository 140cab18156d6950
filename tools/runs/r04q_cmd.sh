#!/bin/bash
# config 5 at HEAD: path selection on the 32-bit keys at LP = 32 (PCG_SEL_K32_LP=32) on the
# interpreter kernel, against the same kernel without (data point for the next round)
set -o pipefail
T=r04q
mkdir -p gpurun_out/$T
timeout -k 10 900 bash tools/sweep_libs.sh scl32 $T/k32 "-|PCG_RTC_SCL=0" "k32lp32|PCG_RTC_SCL=0" || exit 1
