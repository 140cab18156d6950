#!/bin/bash
# Kernel stats + HBM + SQ counters for one bench mode (run on the GPU box via gpurun).
# Usage: bash tools/profile_mode.sh <mode> <tag> <kernel-substring>
set -o pipefail
MODE=${1:-scl8}; TAG=${2:-x}; KS=${3:-scl}
OUT=gpurun_out/prof_${TAG}_${MODE}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --mode $MODE > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python bench.py --mode $MODE --steps 5 --warmup 1 --no-cpu-baseline > $OUT/stats.log 2>&1 || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python bench.py --mode $MODE --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $KS $(find $OUT -name '*counter_collection.csv') > $OUT/summary.txt
cat $OUT/summary.txt
