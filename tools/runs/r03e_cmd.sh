#!/bin/bash
# round-3 evidence step: GPU tests on the in-tree library, then SCL-8 / SCL-32 layout sweeps
set -o pipefail
T=${1:-r03e}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/$T/gputest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/gputest.log | head -20; exit 1; }
timeout -k 10 500 bash tools/sweep_libs.sh scl8 $T "-|PCG_NONE=1" "-|PCG_SCL_SB=8" || exit 1
timeout -k 10 900 bash tools/sweep_libs.sh scl32 $T "-|PCG_NONE=1" "-|PCG_SCL_LDS_KB=30"
