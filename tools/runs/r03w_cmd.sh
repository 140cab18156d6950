#!/bin/bash
# specialised Fast-SSC: lanes per codeword and stored root children re-measured (config 2)
set -o pipefail
timeout -k 10 900 bash tools/sweep_env.sh sc ${1:-r03w} "PCG_NONE=1" "PCG_SCQ_Q=8" "PCG_SCQ_Q=32" "PCG_SCQ_VIRT=0"
