#!/bin/bash
# round 4: exact 4-op F (abs source modifiers), bitop3 G, depuncture fused into the list kernel -- the GPU suite, scl8 / sc / scl32 / nr5g
# rates and the scl8 VALU count
set -o pipefail
T=r04b
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/$T/gputest.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/gputest.log | head -20; exit 1; }
for m in scl8 sc scl32 nr5g; do
  timeout -k 10 300 python bench.py --mode $m --steps 10 --no-cpu-baseline --no-host-rate > gpurun_out/$T/bench_$m.json 2> gpurun_out/$T/bench_$m.err || exit 1
  tail -1 gpurun_out/$T/bench_$m.json | cut -c1-300
done
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES -d gpurun_out/$T/pmc -o run --output-format csv -- python bench.py --mode scl8 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw > gpurun_out/$T/pmc.log 2>&1 || exit 1
python3 tools/pmc_summary.py rtc_kernel $(find gpurun_out/$T/pmc -name "*counter_collection.csv") > gpurun_out/$T/pmc_summary.txt 2>&1; cat gpurun_out/$T/pmc_summary.txt
