#!/bin/bash
# round 4: op profiles of the list kernel at HEAD (SCL-8 config 3, SCL-32 config 5 code) and the
# adaptive decoder's list stage with larger LDS budgets (all stages on chip)
set -o pipefail
T=r04d
mkdir -p gpurun_out/$T
PCG_DEV_LIB=lib_dev/libpcg_ls_prof8.so timeout -k 10 300 python tools/ls_prof.py 8 1024 > gpurun_out/$T/op_profile_scl8.txt 2>&1 || { tail gpurun_out/$T/op_profile_scl8.txt; exit 1; }
cat gpurun_out/$T/op_profile_scl8.txt
PCG_DEV_LIB=lib_dev/libpcg_ls_prof32.so timeout -k 10 300 python tools/ls_prof.py 32 4096 16384 > gpurun_out/$T/op_profile_scl32.txt 2>&1 || { tail gpurun_out/$T/op_profile_scl32.txt; exit 1; }
cat gpurun_out/$T/op_profile_scl32.txt
timeout -k 10 900 bash tools/sweep_libs.sh adaptive8 $T/adapt "-|PCG_NONE=1" "-|PCG_SCL_LDS_KB=160" "-|PCG_SCL_LDS_KB=72" "-|PCG_SCL_LDS_KB=40" || exit 1
