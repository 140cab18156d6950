#!/bin/bash
# round 4 evidence checkpoint: the GPU suite + smoke, then every bench mode (live traffic,
# rocprofv3 kernel stats)
bash tools/round_evidence.sh r04g --tests scl8 sc scl32 nr5g adaptive8 sc_char scl8_char
