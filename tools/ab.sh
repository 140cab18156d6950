#!/bin/bash
# A/B throughput of alternative libpcg builds / env settings in one GPU session.
# Usage: bash tools/ab.sh <mode> 'lib.so[ VAR=val ...]' ...   (each entry run twice, interleaved)
set -o pipefail
MODE=$1; shift
for r in 1 2; do
  for E in "$@"; do
    read -r -a ARR <<< "$E"
    L=${ARR[0]}
    cp "$L" antpolarcodes_amd/lib/libpcg.so || exit 1
    echo -n "$E run$r: "
    env "${ARR[@]:1}" timeout -k 10 300 python bench.py --mode $MODE --no-cpu-baseline --steps 5 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["crc_ok_rate"])' || exit 1
  done
done
