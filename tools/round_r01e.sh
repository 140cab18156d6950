#!/bin/bash
# round-1e evidence: full GPU tests, smoke, bench lines for every mode, rocprof stats + HBM counters
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r01e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for m in scl8 sc scl8_char sc_char adaptive8 nr5g scl32; do
  timeout -k 10 300 python bench.py --mode $m > $OUT/bench_$m.json 2> $OUT/bench_$m.err || { tail -5 $OUT/bench_$m.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$m.json'));print('$m', round(d['value']/1e6,3),'Mcw/s', round(d['roofline']['kernel_ms'],3),'ms', d.get('cpu_baseline',{}).get('value'))"
done
for m in scl8 scl8_char sc_char; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_$m -o run --output-format csv -- python bench.py --mode $m --steps 5 --warmup 1 --no-cpu-baseline > $OUT/stats_$m.log 2>&1 || exit 1
done
for m in scl8_char sc_char; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$m -o run --output-format csv -- python bench.py --mode $m --steps 2 --warmup 1 --no-cpu-baseline > $OUT/fetch_$m.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$m -o run --output-format csv -- python bench.py --mode $m --steps 2 --warmup 1 --no-cpu-baseline > $OUT/write_$m.log 2>&1 || exit 1
done
echo done
