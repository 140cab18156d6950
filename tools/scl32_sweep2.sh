export TMPDIR=/tmp
for w in 0 10 16 24; do
  wpc=""; [ "$w" != 0 ] && wpc="PCG_SCL_WPC=$w"
  env $wpc PCG_DEBUG_OCC=1 timeout -k 10 200 python bench.py --mode scl32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s32.json 2> gpurun_out/s32.err || exit 1
  echo "wpc=$w $(python -c "import json;d=json.load(open('gpurun_out/s32.json'));print(round(d['value']/1e3,1),'kcw/s')") $(grep sclls gpurun_out/s32.err | head -1)"
done
for m in scl8 scl8_char sc sc_char; do
  timeout -k 10 200 python bench.py --mode $m --no-cpu-baseline > gpurun_out/s.json 2>/dev/null || exit 1
  echo "$m $(python -c "import json;d=json.load(open('gpurun_out/s.json'));print(round(d['value']/1e6,2),'Mcw/s')")"
done
