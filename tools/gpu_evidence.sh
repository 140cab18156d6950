#!/bin/bash
# One parametrised GPU evidence run (the command a `gpurun` call executes, from the repository
# root):   bash tools/gpu_evidence.sh <tag> <step> [<step> ...]
# Outputs go to gpurun_out/<tag>/; the summaries worth keeping are copied to profiles/<tag>_*.
# Steps run in order; the first failing step ends the run (nothing more touches the GPU).
#   tests[:<pytest -k expr>]     the GPU suite (or a -k subset) + smoke()
#   bench:<mode>[:<steps>]       bench line (live FETCH/WRITE traffic) + rocprofv3 kernel stats
#   pmc:<mode>                   SQ / TCC / LDS counters of the mode's decode kernel (one pass per group)
#   opprof:<LP>:<N>[:<F>]        per-op cycle profile (needs lib_dev/libpcg_ls_prof<LP>.so, tools/build_dev_lib.sh)
#   sweep:<mode>:<cfg>[;<cfg>..] A/B bench lines, cfg = "<dev lib or ->|VAR=a VAR2=b" (tools/sweep_libs.sh)
#   py:<script> [args]           any python script under tools/ (its stdout to <tag>/py_<n>.txt)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n+1))
  kind=${step%%:*}; arg=${step#*:}; [ "$arg" = "$step" ] && arg=""
  echo "== [$n] $step"
  case $kind in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
          > "$OUT/gputest.log" 2>&1 || { grep -E "Error|assert|FAIL" "$OUT/gputest.log" | head -20; tail -3 "$OUT/gputest.log"; exit 1; }
      tail -1 "$OUT/gputest.log"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
          || { tail -20 "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    bench)
      MODE=${arg%%:*}; STEPS=10; [ "$MODE" != "$arg" ] && STEPS=${arg##*:}
      bash tools/profile_mode.sh "$MODE" "$TAG" "$STEPS" || { echo "bench $MODE failed"; tail -5 "$OUT/$MODE.err"; exit 1; }
      python3 -c "
import json; d=json.loads(open('$OUT/$MODE.json').read().splitlines()[-1]); r=d['roofline']
print('$MODE', '%.4g' % d['value'], r['kernel'], 'ms %.3f' % r['kernel_ms'], 'frac %.4f' % r['frac'],
      'traffic/cw', r.get('traffic_bytes_per_codeword'), r.get('traffic_note') or '',
      'host %.3g' % d.get('host_buffers_cw_per_s', 0), 'cpu', d.get('cpu_baseline', {}).get('value'))" ;;
    pmc)
      timeout -k 10 600 bash tools/pmc_scl8.sh "$arg" "$TAG/pmc_$arg" || exit 1 ;;
    opprof)
      IFS=: read -r LP N F <<< "$arg"
      PCG_DEV_LIB=lib_dev/libpcg_ls_prof$LP.so timeout -k 10 400 python tools/ls_prof.py "$LP" "$N" ${F:+"$F"} \
          > "$OUT/op_profile_lp$LP.txt" 2>&1 || { tail "$OUT/op_profile_lp$LP.txt"; exit 1; }
      cat "$OUT/op_profile_lp$LP.txt" ;;
    sweep)
      MODE=${arg%%:*}; CFGS=${arg#*:}
      IFS=';' read -r -a C <<< "$CFGS"
      timeout -k 10 1000 bash tools/sweep_libs.sh "$MODE" "$TAG/sweep_$n" "${C[@]}" || exit 1 ;;
    py)
      # shellcheck disable=SC2086
      timeout -k 10 600 python $arg > "$OUT/py_$n.txt" 2>&1 || { tail -20 "$OUT/py_$n.txt"; exit 1; }
      tail -30 "$OUT/py_$n.txt" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
