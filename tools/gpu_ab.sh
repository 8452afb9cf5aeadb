#!/bin/bash
# A/B timing of kernel variants: GPU tests (default variant), then one short headline
# bench per value of $VAR in $VALS.  Usage: TAG=x VAR=XT_W_VARIANT VALS="1 2" tools/gpu_ab.sh
# VAR=ENV: each value is a comma-separated list of assignments (VALS="A=0,B=1 A=1,B=1")
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc = 0 ] || exit $rc
fi
for v in ${VALS:-0}; do
  if [ "${VAR:-}" = ENV ]; then asg=$(echo "$v" | tr "," " "); else asg="${VAR:-XT_NONE}=$v"; fi
  env $asg timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-converge ${BENCH_ARGS:-} > "$OUT/b_$v.log" 2>&1
  rc=$?; [ $rc = 0 ] || { tail -5 "$OUT/b_$v.log"; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: v['ms_per_step'] for k, v in d['gemm_classes'].items()})" "$OUT/b_$v.log" "$v"
done
