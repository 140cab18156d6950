#!/bin/bash
# round 4 evidence: the GPU suite + smoke, every bench mode (live traffic, rocprof stats), the
# SCL-8 PMC counters and op profile, the 8-bit specialised kernels' A/B
set -o pipefail
T=r04j
mkdir -p gpurun_out/$T
bash tools/round_evidence.sh $T --tests scl8 sc scl32 nr5g adaptive8 sc_char scl8_char adaptive8_char || exit 1
timeout -k 10 400 bash tools/pmc_scl8.sh scl8 $T/pmc || exit 1
PCG_DEV_LIB=lib_dev/libpcg_ls_prof8.so timeout -k 10 300 python tools/ls_prof.py 8 1024 > gpurun_out/$T/op_profile_scl8.txt 2>&1 || { tail gpurun_out/$T/op_profile_scl8.txt; exit 1; }
cat gpurun_out/$T/op_profile_scl8.txt
timeout -k 10 600 bash tools/sweep_libs.sh scl8_char $T/char "-|PCG_NONE=1" "-|PCG_RTC=0" || exit 1
timeout -k 10 900 bash tools/sweep_libs.sh scl32 $T/wk32 "-|PCG_NONE=1" "wk32|PCG_NONE=1" || exit 1
