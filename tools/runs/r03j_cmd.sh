#!/bin/bash
# SCL-32 op profile (LP=32 profiling build) + PMC passes of the config-5 shard
set -o pipefail
T=${1:-r03j}
mkdir -p gpurun_out/$T
PCG_DEV_LIB=lib_dev/libpcg_ls_prof32.so timeout -k 10 300 python tools/ls_prof.py 32 4096 16384 > gpurun_out/$T/prof32.txt 2>&1 || { tail -5 gpurun_out/$T/prof32.txt; exit 1; }
cat gpurun_out/$T/prof32.txt
timeout -k 10 600 bash tools/pmc_scl8.sh scl32 $T
