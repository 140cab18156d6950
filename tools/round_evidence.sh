#!/bin/bash
# Round evidence on the GPU box: [tests] then bench line (live traffic) + rocprofv3 kernel
# stats per mode.  Usage: bash tools/round_evidence.sh <tag> [--tests] mode[:steps] ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$1" == "--tests" ]; then
  shift
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -20 $OUT/gputest.log; exit 1; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/gputest.log; tail -1 $OUT/smoke.log
fi
for ms in "$@"; do
  MODE=${ms%%:*}; STEPS=10
  [ "$ms" != "$MODE" ] && STEPS=${ms##*:}
  bash tools/profile_mode.sh $MODE $TAG $STEPS || { echo "profile $MODE failed"; tail -5 $OUT/$MODE.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$OUT/$MODE.json').read().splitlines()[-1]); r=d['roofline']
print('$MODE', '%.4g' % d['value'], r['kernel'], 'ms %.3f' % r['kernel_ms'], 'frac %.4f' % r['frac'], 'traffic/cw', r.get('traffic_bytes_per_codeword'), r.get('traffic_note'), 'cpu', d.get('cpu_baseline',{}).get('value'))"
done
