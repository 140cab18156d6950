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
# the same steps under the kernel tracer (one stream): its bench line is kept, so the trace's
# average over the timed launches can be checked against that run's own HIP-event time and
# against the unprofiled line above (tools/reconcile_profile.py)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/${MODE}_stats -o run --output-format csv -- \
    python bench.py --mode $MODE --steps $STEPS --warmup 2 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw --no-in-flight \
    > $OUT/${MODE}_stats.log 2>&1 || exit 1
grep '^{' $OUT/${MODE}_stats.log | tail -1 > $OUT/${MODE}_profiled.json
KER=$(python3 -c "import json; print(json.loads(open('$OUT/${MODE}_profiled.json').read())['roofline']['kernel'])")
python3 tools/reconcile_profile.py $OUT/${MODE}_stats/run_kernel_trace.csv "$KER" 2 $OUT/${MODE}_profiled.json $OUT/$MODE.json \
    > $OUT/${MODE}_reconcile.txt 2>&1 || true
