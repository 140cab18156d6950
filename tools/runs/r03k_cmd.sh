#!/bin/bash
# quarters recomputed (PCG_SCL_VIRT=2): GPU suite under the switch, then SCL-8 / SCL-32 / nr5g A/B
set -o pipefail
T=${1:-r03k}
mkdir -p gpurun_out/$T
PCG_SCL_VIRT=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gputest_v2.log 2>&1
rc=$?; tail -2 gpurun_out/$T/gputest_v2.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/gputest_v2.log | head -20; exit 1; }
timeout -k 10 500 bash tools/sweep_libs.sh scl8 $T "-|PCG_NONE=1" "-|PCG_SCL_VIRT=2" || exit 1
timeout -k 10 500 bash tools/sweep_libs.sh nr5g $T "-|PCG_NONE=1" "-|PCG_SCL_VIRT=2" || exit 1
timeout -k 10 600 bash tools/sweep_libs.sh scl32 $T "-|PCG_NONE=1" "-|PCG_SCL_VIRT=2"
