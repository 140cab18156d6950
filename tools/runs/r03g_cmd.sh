set -o pipefail
mkdir -p gpurun_out/r03g
PCG_DEV_LIB=lib_dev/libpcg_ls_prof.so timeout -k 10 200 python tools/ls_prof.py 8 > gpurun_out/r03g/prof_new.txt 2>&1 || exit 1
PCG_DEV_LIB=lib_dev/libpcg_old_prof.so timeout -k 10 200 python tools/ls_prof.py 8 > gpurun_out/r03g/prof_old.txt 2>&1 || exit 1
paste gpurun_out/r03g/prof_old.txt gpurun_out/r03g/prof_new.txt
timeout -k 10 400 bash tools/sweep_libs.sh scl8 r03g "old8|PCG_NONE=1" "-|PCG_NONE=1"
