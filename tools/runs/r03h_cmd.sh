#!/bin/bash
# GPU tests, SCL-8 op profile, SCL-8 / SCL-32 bench lines
set -o pipefail
T=${1:-r03h}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/$T/gputest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/gputest.log | head -20; exit 1; }
PCG_DEV_LIB=lib_dev/libpcg_ls_prof.so timeout -k 10 200 python tools/ls_prof.py 8 > gpurun_out/$T/prof8.txt 2>&1 || exit 1
cat gpurun_out/$T/prof8.txt
timeout -k 10 400 bash tools/sweep_libs.sh scl8 $T "-|PCG_NONE=1" || exit 1
timeout -k 10 600 bash tools/sweep_libs.sh scl32 $T "-|PCG_NONE=1"
