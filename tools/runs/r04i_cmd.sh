#!/bin/bash
# round 4: SCL-8 op profile at HEAD (32-bit-key selection and weak search)
set -o pipefail
T=r04i
mkdir -p gpurun_out/$T
PCG_DEV_LIB=lib_dev/libpcg_ls_prof8.so timeout -k 10 300 python tools/ls_prof.py 8 1024 > gpurun_out/$T/op_profile_scl8.txt 2>&1 || { tail gpurun_out/$T/op_profile_scl8.txt; exit 1; }
cat gpurun_out/$T/op_profile_scl8.txt
# the 8-bit decoders' specialised kernels: parity and rates
timeout -k 10 600 python -u -m pytest tests/test_gpu_char.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/char_test.log 2>&1
rc=$?; tail -2 gpurun_out/$T/char_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/char_test.log | head -20; exit 1; }
timeout -k 10 600 bash tools/sweep_libs.sh scl8_char $T/char "-|PCG_NONE=1" "-|PCG_RTC=0" || exit 1
timeout -k 10 600 bash tools/sweep_libs.sh adaptive8_char $T/char "-|PCG_NONE=1" "-|PCG_RTC=0" || exit 1
