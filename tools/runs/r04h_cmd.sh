#!/bin/bash
# round 4: 32-bit-key selection (LP <= 8) and weak-LLR search -- the GPU suite + smoke, the list
# modes' bench lines with rocprof stats, the SCL-8 PMC counters
set -o pipefail
bash tools/round_evidence.sh r04h --tests scl8 scl32 nr5g adaptive8 || exit 1
timeout -k 10 400 bash tools/pmc_scl8.sh scl8 r04h/pmc || exit 1
