#!/bin/bash
# config 5 (LP = 32) at HEAD, for the next round's ranking: the op profile (interpreter build
# with PCG_LS_PROF), the ablation bounds of path selection and the weak-LLR search (interpreter
# kernel, wrong results by design: cost measurement only), and the SQ/TCC counters
set -o pipefail
T=r04p
mkdir -p gpurun_out/$T
PCG_DEV_LIB=lib_dev/libpcg_ls_prof32.so timeout -k 10 400 python tools/ls_prof.py 32 4096 32768 > gpurun_out/$T/op_profile_scl32.txt 2>&1 || { tail gpurun_out/$T/op_profile_scl32.txt; exit 1; }
cat gpurun_out/$T/op_profile_scl32.txt
timeout -k 10 900 bash tools/sweep_libs.sh scl32 $T/abl "-|PCG_RTC_SCL=0" "abl_sel32|PCG_RTC_SCL=0" "abl_weak32|PCG_RTC_SCL=0" || exit 1
timeout -k 10 600 bash tools/pmc_scl8.sh scl32 $T/pmc || exit 1
