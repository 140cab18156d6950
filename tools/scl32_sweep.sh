export TMPDIR=/tmp
for cfg in "20 0" "12 0" "32 0" "48 0" "20 4" "20 12" "12 16"; do
  set -- $cfg
  wpc=""; [ "$2" != 0 ] && wpc="PCG_SCL_WPC=$2"
  env $wpc PCG_SCL_LDS_KB=$1 PCG_DEBUG_OCC=1 timeout -k 10 200 python bench.py --mode scl32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s32.json 2> gpurun_out/s32.err || exit 1
  echo "kb=$1 wpc=$2 $(python -c "import json;d=json.load(open('gpurun_out/s32.json'));print(round(d['value']/1e3,1),'kcw/s', d['frame_error_rate'])") $(grep sclls gpurun_out/s32.err | head -1)"
done
