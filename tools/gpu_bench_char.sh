set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --mode sc_char > gpurun_out/bench_sc_char.json 2> gpurun_out/bench_sc_char.err &&
timeout -k 10 300 python bench.py --mode scl8_char > gpurun_out/bench_scl8_char.json 2> gpurun_out/bench_scl8_char.err &&
PCG_DEBUG_OCC=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_char -o run -- python3 bench.py --mode scl8_char --steps 5 --no-cpu-baseline > gpurun_out/prof_char.log 2>&1
