# char SCL: parity, then a layout sweep of the bench (run on the GPU box via gpurun)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_char.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sweep_tests.log 2>&1 || { tail -20 gpurun_out/sweep_tests.log; exit 1; }
for kb in ${KBS:-16 20 24 28 40 64}; do
  PCG_SCLC_LDS_KB=$kb PCG_DEBUG_OCC=1 timeout -k 10 120 python bench.py --mode scl8_char --no-cpu-baseline > gpurun_out/sweep_$kb.json 2> gpurun_out/sweep_$kb.err || exit 1
  echo "kb=$kb $(python -c "import json;d=json.load(open('gpurun_out/sweep_$kb.json'));print(round(d['value']/1e6,2),'Mcw/s', round(d['roofline']['kernel_ms'],3),'ms')") $(grep sclc gpurun_out/sweep_$kb.err | head -1)"
done
