#!/bin/bash
# GPU suite at the default (quarters recomputed where allowed), then A/B against virt = 1
set -o pipefail
T=${1:-r03l}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
rc=$?; tail -2 gpurun_out/$T/gputest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/gputest.log | head -20; exit 1; }
timeout -k 10 500 bash tools/sweep_libs.sh scl8 $T "-|PCG_NONE=1" "-|PCG_SCL_VIRT=1" || exit 1
timeout -k 10 500 bash tools/sweep_libs.sh nr5g $T "-|PCG_NONE=1" "-|PCG_SCL_VIRT=1" || exit 1
timeout -k 10 600 bash tools/sweep_libs.sh scl32 $T "-|PCG_NONE=1"
