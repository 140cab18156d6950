#!/bin/bash
# Run on the GPU box (via gpurun): bench lines + rocprofv3 kernel stats + HBM counters.
# Usage: bash tools/profile_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_scl8.json 2> $OUT/bench_scl8.err || exit 1
timeout -k 10 300 python bench.py --mode sc --no-cpu-baseline > $OUT/bench_sc.json 2> $OUT/bench_sc.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/sq -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/sq.log 2>&1 || exit 1
echo done
