#!/bin/bash
# Kernel-variant A/B in one GPU call: optional parity tests per variant, then one
# short headline bench per variant.  VARIANTS: ';'-separated env assignments
# (e.g. "XT_M_MAP=0;XT_M_MAP=1;XT_W_BN=128"), "-" for the defaults.
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-var}
mkdir -p "$OUT"
IFS=';' read -ra VS <<< "${VARIANTS:--}"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  [ "$v" = "-" ] && v="XT_NONE=1"
  if [ -n "${TESTS:-}" ]; then
    env $v timeout -k 10 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > "$OUT/t_$i.log" 2>&1
    rc=$?; echo "[$v] tests: $(tail -1 "$OUT/t_$i.log")"; [ $rc = 0 ] || exit $rc
  fi
  env $v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-converge ${BENCH_ARGS:-} > "$OUT/b_$i.log" 2>&1
  rc=$?; [ $rc = 0 ] || { echo "[$v] bench failed"; tail -5 "$OUT/b_$i.log"; exit $rc; }
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], {k: v['ms_per_step'] for k, v in d['gemm_classes'].items()}, flush=True)" "$OUT/b_$i.log" "[$v]"
done
