#!/bin/bash
# FETCH_SIZE of the duplicate-address probe, one rocprofv3 pass per pattern (gpurun_out/<tag>/).
set -o pipefail
OUT=gpurun_out/${1:-dup}
mkdir -p $OUT
export TMPDIR=/tmp
for p in 0 1 2 3; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/p$p -o run --output-format csv -- ./tools/probes/dup_fetch_probe $p \
      > $OUT/p$p.log 2>&1 || { tail -5 $OUT/p$p.log; exit 1; }
  grep pattern $OUT/p$p.log
  python3 - "$OUT/p$p" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "probe" in r.get("Kernel_Name", "")]
by = {}
for r in rows:
    by.setdefault(r["Dispatch_Id"], 0.0)
    by[r["Dispatch_Id"]] += float(r["Counter_Value"])
for d, v in sorted(by.items(), key=lambda x: int(x[0])):
    print(f"  dispatch {d}: FETCH_SIZE {v:.4g} (x1024 B = {v * 1024:.4g} B; gfx950 16-B/lane reads x2 = {2 * v * 1024:.4g} B)")
PY
done
