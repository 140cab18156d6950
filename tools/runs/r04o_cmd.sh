#!/bin/bash
# round-4 closing evidence at HEAD: the GPU suite + smoke, every bench mode (live traffic,
# rocprof stats), the SCL-8 PMC counters
set -o pipefail
T=r04o
mkdir -p gpurun_out/$T
bash tools/round_evidence.sh $T --tests scl8 sc scl32 nr5g adaptive8 sc_char scl8_char adaptive8_char || exit 1
timeout -k 10 400 bash tools/pmc_scl8.sh scl8 $T/pmc || exit 1
