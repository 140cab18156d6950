#!/bin/bash
set -o pipefail
T=${1:-r03n}
timeout -k 10 900 bash tools/round_evidence.sh $T --tests scl8 scl32:3 nr5g adaptive8 || exit 1
timeout -k 10 500 bash tools/sweep_libs.sh scl8_char $T "-|PCG_NONE=1" "-|PCG_SCLC_LDS_KB=16" "-|PCG_SCLC_LDS_KB=24"
