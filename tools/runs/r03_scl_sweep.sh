#!/bin/bash
# Round-3 SCL experiments on one GPU box call: live-traffic bench lines for scl8 under the
# layout switches the verdict asked about (lanes per codeword, resident waves, LDS budget,
# recomputed stages), then the HEAD per-op cycle profiles of scl8 and scl32 (labelled
# buckets, tools/ls_prof.py with the -DPCG_LS_PROF variant in lib_dev/).
set -o pipefail
TAG=${1:-r03_sweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/sweep_env.sh scl8 $TAG "PCG_NONE=1" "PCG_SCL_VIRT=2" "PCG_SCL_LP=16" "PCG_SCL_WPC=5" "PCG_SCL_WPC=6" \
    "PCG_SCL_LDS_KB=16" "PCG_SCL_LDS_KB=32" || exit 1
PCG_DEV_LIB=lib_dev/libpcg_ls_prof.so timeout -k 10 300 python tools/ls_prof.py 8 1024 > $OUT/ls_prof_scl8.txt 2>&1 || exit 1
PCG_DEV_LIB=lib_dev/libpcg_ls_prof.so timeout -k 10 300 python tools/ls_prof.py 32 4096 32768 > $OUT/ls_prof_scl32.txt 2>&1 || exit 1
cat $OUT/ls_prof_scl8.txt $OUT/ls_prof_scl32.txt
