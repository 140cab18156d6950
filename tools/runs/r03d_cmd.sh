set -o pipefail
mkdir -p gpurun_out/r03d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/gputest.log 2>&1; rc=$?; tail -2 gpurun_out/r03d/gputest.log; [ $rc -eq 0 ] || exit 1
PCG_DEV_LIB=lib_dev/libpcg_sqw.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sc.py tests/test_gpu_soft.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03d/sqw_test.log 2>&1; rc=$?; tail -1 gpurun_out/r03d/sqw_test.log; [ $rc -eq 0 ] || exit 1
PCG_SCL_V3=2 timeout -k 10 300 python tools/scl8_parity_quick.py || exit 1
PCG_SCL_V3=2 PCG_DEV_LIB=lib_dev/libpcg_w3.so timeout -k 10 300 python tools/scl8_parity_quick.py || exit 1
timeout -k 10 400 bash tools/sweep_libs.sh sc r03d "-|PCG_NONE=1" "sqw|PCG_NONE=1" "sqw|PCG_SCQ_WPC=12" || exit 1
timeout -k 10 700 bash tools/sweep_libs.sh scl8 r03d "-|PCG_NONE=1" "-|PCG_SCL_V3=2" "w3|PCG_SCL_V3=2" "w3|PCG_SCL_V3=1" "w3|PCG_SCL_V3=2 PCG_SCL_WPC=9"
