set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_char.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sccs_tests.log 2>&1 || { tail -30 gpurun_out/sccs_tests.log; exit 1; }
tail -1 gpurun_out/sccs_tests.log
for kb in ${KBS:-12 16 24 40}; do
  PCG_SCCS_LDS_KB=$kb PCG_DEBUG_OCC=1 timeout -k 10 120 python bench.py --mode sc_char --no-cpu-baseline > gpurun_out/sccs_$kb.json 2> gpurun_out/sccs_$kb.err || exit 1
  echo "kb=$kb $(python -c "import json;d=json.load(open('gpurun_out/sccs_$kb.json'));print(round(d['value']/1e6,2),'Mcw/s', round(d['roofline']['kernel_ms'],3),'ms fer', d['frame_error_rate'])") $(grep sccs gpurun_out/sccs_$kb.err | head -1)"
done
