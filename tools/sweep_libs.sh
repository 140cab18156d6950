#!/bin/bash
# Bench one mode with several dev libraries / environment settings, one JSON line each with
# live traffic.  Usage: bash tools/sweep_libs.sh <mode> <tag> "LIB|VAR=a VAR2=b" ...
#   LIB: a lib_dev/libpcg_<LIB>.so variant (tools/build_dev_lib.sh) or "-" for the in-tree one
set -o pipefail
MODE=$1; TAG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  lib=${cfg%%|*}; envs=${cfg#*|}
  dl=""
  [ "$lib" != "-" ] && dl="PCG_DEV_LIB=lib_dev/libpcg_$lib.so"
  echo "== $cfg" >> $OUT/sweep_$MODE.txt
  env $dl $envs timeout -k 10 300 python bench.py --mode $MODE --steps 10 --no-cpu-baseline --no-host-rate --no-copy-bw --no-in-flight \
      > $OUT/sweep_${MODE}_$i.json 2> $OUT/sweep_${MODE}_$i.err || exit 1
  python3 -c "
import json,sys
d=json.loads(open('$OUT/sweep_${MODE}_$i.json').read().splitlines()[-1]); r=d['roofline']
print('$cfg', '%.4g cw/s' % d['value'], 'kernel_ms %.3f' % r['kernel_ms'], 'traffic/cw', r.get('traffic_bytes_per_codeword'), 'R', r.get('traffic_read_bytes_per_codeword'), 'W', r.get('traffic_write_bytes_per_codeword'), 'fer', d.get('frame_error_rate'))
" >> $OUT/sweep_$MODE.txt
done
cat $OUT/sweep_$MODE.txt
