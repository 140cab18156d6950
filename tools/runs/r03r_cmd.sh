#!/bin/bash
# plan-specialised scq kernel: parity (config 2) + interpreter refactor parity + sc bench A/B
set -o pipefail
T=${1:-r03r}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sc.py tests/test_gpu_soft.py tests/test_gpu_rtc.py::test_rtc_auto_large_batch_config2 -x -q --timeout 300 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/test.log | head; exit 1; }
for v in 0 2; do
  PCG_RTC=$v timeout -k 10 300 python bench.py --mode sc --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw > $O/sc_rtc$v.json 2> $O/sc_rtc$v.err || { tail -5 $O/sc_rtc$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sc_rtc$v.json').read().splitlines()[-1]); print('PCG_RTC=$v', '%.4g' % d['value'], d['roofline']['kernel'], 'ms %.4f' % d['roofline']['kernel_ms'])"
done
