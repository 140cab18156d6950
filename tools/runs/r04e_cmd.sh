#!/bin/bash
# round 4: ablation bounds on the SCL-8 interpreter kernel (wrong results by design: the cost of
# path selection and of the weak-LLR search), with the VALU count of each; the value-merge
# selection (PCG_SEL_VMERGE=1) for parity and rate
set -o pipefail
T=r04e
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
for L in 8 6; do
  PCG_RTC=0 PCG_DEV_LIB=lib_dev/libpcg_vm1.so timeout -k 10 300 python tools/scl8_parity_quick.py $L > gpurun_out/$T/vm1_parity_L$L.txt 2>&1 || { tail gpurun_out/$T/vm1_parity_L$L.txt; exit 1; }
  tail -2 gpurun_out/$T/vm1_parity_L$L.txt
done
timeout -k 10 900 bash tools/sweep_libs.sh scl8 $T/abl "-|PCG_RTC_SCL=0" "abl_sel|PCG_RTC_SCL=0" "abl_weak|PCG_RTC_SCL=0" "vm1|PCG_RTC_SCL=0" "-|PCG_NONE=1" "vm1|PCG_NONE=1" || exit 1
i=0
for lib in "" lib_dev/libpcg_abl_sel.so lib_dev/libpcg_abl_weak.so lib_dev/libpcg_vm1.so; do
  i=$((i+1))
  env ${lib:+PCG_DEV_LIB=$lib} PCG_RTC_SCL=0 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH -d gpurun_out/$T/pmc$i -o run --output-format csv -- python bench.py --mode scl8 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw > gpurun_out/$T/pmc$i.log 2>&1 || exit 1
  echo "== ${lib:-in-tree}"; python3 tools/pmc_summary.py sclls_kernel $(find gpurun_out/$T/pmc$i -name "*counter_collection.csv")
done | tee gpurun_out/$T/pmc_summary.txt
# the 8-bit Fast-SSC decoder's specialised kernel: parity and rate
timeout -k 10 600 python -u -m pytest tests/test_gpu_char.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$T/char_test.log 2>&1
rc=$?; tail -2 gpurun_out/$T/char_test.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/$T/char_test.log | head -20; exit 1; }
timeout -k 10 600 bash tools/sweep_libs.sh sc_char $T/char "-|PCG_NONE=1" "-|PCG_RTC=0" || exit 1
