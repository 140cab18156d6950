set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_char.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_char.log 2>&1
