#!/bin/bash
set -o pipefail
T=${1:-r03p}
mkdir -p gpurun_out/$T
PCG_DEV_LIB=lib_dev/libpcg_scqdpp.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sc.py tests/test_gpu_soft.py tests/test_gpu_adaptive.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/scq_test.log 2>&1
rc=$?; tail -1 gpurun_out/$T/scq_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/scq_test.log | head; exit 1; }
timeout -k 10 400 bash tools/sweep_libs.sh sc $T "-|PCG_NONE=1" "scqdpp|PCG_NONE=1" || exit 1
timeout -k 10 400 bash tools/sweep_libs.sh adaptive8 $T "-|PCG_NONE=1" "-|PCG_SCL_VIRT=1"
