#!/bin/bash
# SQ / TCC counters of one bench mode's decode kernel, one rocprofv3 --pmc pass per counter
# group (the guide's per-block limits), each pass its own run under a hard time limit.
#   bash tools/pmc_scl8.sh <mode> <tag> [PCG_DEV_LIB=...]
set -o pipefail
MODE=${1:-scl8}; TAG=${2:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$3" ] && export $3
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" \
           "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- \
      python bench.py --mode $MODE --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-host-rate --no-copy-bw --no-in-flight \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'EOF'
import csv, glob, collections, sys
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in ("sclls_kernel", "scq_kernel", "scl_char", "rtc_kernel", "sccs_kernel")):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(out + "/pmc_summary.txt", "w") as fh:
    for k, v in sorted(agg.items()):
        v.sort()
        line = f"{k:28s} n={len(v):3d} median={v[len(v)//2]:.6g}"
        print(line)
        fh.write(line + "\n")
EOF
