#!/bin/bash
# round 4: PC sampling of the SCL-8 list kernel (which instructions the waves sit on)
set -o pipefail
T=r04c
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/$T/list_avail.txt 2>&1
grep -i -A12 "pc.sampl\|PC_SAMPL\|method" gpurun_out/$T/list_avail.txt | head -60
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/$T/pcs -o run --output-format csv -- python bench.py --mode scl8 --steps 3 --warmup 1 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw > gpurun_out/$T/pcs.log 2>&1
echo "rc=$?"; tail -5 gpurun_out/$T/pcs.log; find gpurun_out/$T/pcs -type f | head; ls -la $(find gpurun_out/$T/pcs -type f) | head
