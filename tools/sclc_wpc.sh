export TMPDIR=/tmp
for w in 8 10 12 14; do
  PCG_SCLC_WPC=$w timeout -k 10 120 python bench.py --mode scl8_char --no-cpu-baseline > gpurun_out/wpc_$w.json 2>/dev/null || exit 1
  echo "wpc=$w $(python -c "import json;d=json.load(open('gpurun_out/wpc_$w.json'));print(round(d['value']/1e6,2),'Mcw/s')")"
done
for kb in 12 16; do for L in 4 16 32; do
  PCG_SCLC_LDS_KB=$kb timeout -k 10 120 python tools/quick_bench.py --L $L --reps 5 > /dev/null 2>&1 || true
done; done
