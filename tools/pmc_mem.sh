#!/bin/bash
# L2 / L1 memory-system counters for the SCL bench kernel (run on the GPU box via gpurun).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcm_${1:-x}
mkdir -p $OUT
i=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_WRITE_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCC_TAG_STALL_sum" \
           "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/p$i -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
python tools/pmc_summary.py scl $(find $OUT -name '*counter_collection.csv')
