#!/bin/bash
# list plans with literal layout / plan constants (PCG_RTC_SCL=1, loop kept): parity + scl8 / scl32 A/B
set -o pipefail
T=${1:-r03t}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
PCG_RTC=1 PCG_RTC_SCL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_scl.py -k "config3 or config5_shard or crc_and_systematic" -x -q --timeout 400 --timeout-method thread > $O/test.log 2>&1
rc=$?; tail -2 $O/test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/test.log | head; exit 1; }
for m in scl8 scl32; do
  st=20; [ $m == scl32 ] && st=3
  for v in 0 1; do
    PCG_RTC_SCL=$v timeout -k 10 400 python bench.py --mode $m --steps $st --warmup 2 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw > $O/${m}_$v.json 2> $O/${m}_$v.err || { tail -5 $O/${m}_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${m}_$v.json').read().splitlines()[-1]); print('$m PCG_RTC_SCL=$v', '%.4g' % d['value'], d['roofline']['kernel'], 'ms %.4f' % d['roofline']['kernel_ms'], 'fer', d['frame_error_rate'])"
  done
done
