export TMPDIR=/tmp
for m in m3 m4; do
  for wpc in 8 12 16; do
    PCG_DEV_LIB=altlib/libpcg_$m.so PCG_SCL_WPC=$wpc PCG_DEBUG_OCC=1 timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/minw_$m_$wpc.json 2> gpurun_out/minw.err || exit 1
    echo "$m wpc=$wpc $(python -c "import json;d=json.load(open('gpurun_out/minw_$m_$wpc.json'));print(round(d['value']/1e6,2),'Mcw/s', d['frame_error_rate'])") $(grep sclls gpurun_out/minw.err | head -1)"
  done
done
