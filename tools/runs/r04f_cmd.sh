#!/bin/bash
# round 4: 32-bit-key bitonic selection (PCG_SEL_K32) on the SCL-8 interpreter kernel: parity
# (quick oracle sweep, L = 8 and 6) and rate / VALU against the 64-bit selection
set -o pipefail
T=r04f
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for L in 8 6 5; do
  PCG_RTC=0 PCG_DEV_LIB=lib_dev/libpcg_k32.so timeout -k 10 300 python tools/scl8_parity_quick.py $L > gpurun_out/$T/k32_parity_L$L.txt 2>&1 || { tail gpurun_out/$T/k32_parity_L$L.txt; exit 1; }
  tail -1 gpurun_out/$T/k32_parity_L$L.txt
done
timeout -k 10 600 bash tools/sweep_libs.sh scl8 $T/ab "-|PCG_RTC_SCL=0" "k32|PCG_RTC_SCL=0" || exit 1
i=0
for lib in "" lib_dev/libpcg_k32.so; do
  i=$((i+1))
  env ${lib:+PCG_DEV_LIB=$lib} PCG_RTC_SCL=0 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH -d gpurun_out/$T/pmc$i -o run --output-format csv -- python bench.py --mode scl8 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw > gpurun_out/$T/pmc$i.log 2>&1 || exit 1
  echo "== ${lib:-in-tree}"; python3 tools/pmc_summary.py sclls_kernel $(find gpurun_out/$T/pmc$i -name "*counter_collection.csv")
done | tee gpurun_out/$T/pmc_summary.txt
