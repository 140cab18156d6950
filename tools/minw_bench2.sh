export TMPDIR=/tmp
for cfg in "m3 12 12" "m3 14 12" "m4 12 16" "m4 10 16" "base 12 8" "base 16 8"; do
  set -- $cfg
  lib=""; [ "$1" != base ] && lib="PCG_DEV_LIB=altlib/libpcg_$1.so"
  env $lib PCG_SCL_LDS_KB=$2 PCG_SCL_WPC=$3 PCG_DEBUG_OCC=1 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/mw.json 2> gpurun_out/mw.err || exit 1
  echo "$cfg $(python -c "import json;d=json.load(open('gpurun_out/mw.json'));print(round(d['value']/1e6,2),'Mcw/s', d['frame_error_rate'])") $(grep sclls gpurun_out/mw.err | head -1)"
done
