#!/bin/bash
# GPU suite + smoke + scl32 at HEAD (weak-LLR search on 32-bit keys at every width), then
# config 5 with one wave per SIMD (PCG_LS_MINW=1: no scratch spills) at 20 / 40 KB LDS per wave
set -o pipefail
T=r04k
mkdir -p gpurun_out/$T
bash tools/round_evidence.sh $T --tests scl32 || exit 1
timeout -k 10 900 bash tools/sweep_libs.sh scl32 $T/minw "-|PCG_NONE=1" "minw1_32|PCG_RTC_CACHE=lib_dev/rtc" \
    "minw1_32|PCG_RTC_CACHE=lib_dev/rtc PCG_SCL_LDS_KB=40" || exit 1
bash tools/runs/r04l_cmd.sh || exit 1
