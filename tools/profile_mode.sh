#!/bin/bash
# Bench line (with live FETCH/WRITE traffic) + rocprofv3 kernel stats for one bench mode,
# run on the GPU box via gpurun.  Usage: bash tools/profile_mode.sh <mode> <tag> [steps]
# Writes gpurun_out/<tag>/<mode>.json (bench line) and gpurun_out/<tag>/<mode>_stats/.
set -o pipefail
MODE=${1:-scl8}; TAG=${2:-x}; STEPS=${3:-10}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --mode $MODE --steps $STEPS > $OUT/$MODE.json 2> $OUT/$MODE.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${MODE}_stats -o run --output-format csv -- \
    python bench.py --mode $MODE --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw --no-in-flight \
    > $OUT/${MODE}_stats.log 2>&1 || exit 1
