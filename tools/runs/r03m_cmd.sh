#!/bin/bash
set -o pipefail
T=${1:-r03m}
timeout -k 10 900 bash tools/round_evidence.sh $T --tests scl8 scl32:3 nr5g adaptive8 sc || exit 1
timeout -k 10 300 bash tools/pmc_scl8.sh sc $T
