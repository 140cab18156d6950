#!/bin/bash
# specialised list plans by default: the rtc tests, then the round evidence (all GPU tests + benches)
set -o pipefail
T=${1:-r03v}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_rtc.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/rtc_test.log 2>&1
rc=$?; tail -1 gpurun_out/$T/rtc_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/rtc_test.log | head; exit 1; }
bash tools/round_evidence.sh $T --tests scl8 scl32:3
