export TMPDIR=/tmp
for m in scl8 scl8_char sc sc_char scl32; do
  for w in 0 16 32; do
    wpc=""; [ "$w" != 0 ] && wpc="PCG_SCL_WPC=$w PCG_SCLC_WPC=$w PCG_SCS_WPC=$w PCG_SCCS_WPC=$w"
    env $wpc timeout -k 10 200 python bench.py --mode $m --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/o.json 2>/dev/null || exit 1
    echo "$m wpc=$w $(python -c "import json;d=json.load(open('gpurun_out/o.json'));print(round(d['value']/1e6,3),'Mcw/s')")"
  done
done
