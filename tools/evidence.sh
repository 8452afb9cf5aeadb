#!/bin/bash
# Round evidence per bench configuration, in one GPU call (run from the repo root):
#   for each config in CONFIGS (default "H"):
#     1) the full bench line (CPU baseline + Davidson convergence included)
#     2) rocprofv3 --kernel-trace --stats of a short bench run
#     3) PMC FETCH_SIZE pass, 4) PMC WRITE_SIZE pass (separate passes,
#        MI355X_MICROARCH.md HBM section), each under its own time limit
# Summarise afterwards with  python tools/parse_prof.py gpurun_out/<TAG> r02
#   CONFIGS  space-separated bench configs      SKIP_BENCH=1  profiles only
#   PMC=0    skip the counter passes
set -uo pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-evidence}
mkdir -p "$OUT"
for c in ${CONFIGS:-H}; do
  D="$OUT/$c"
  mkdir -p "$D"
  if [ -z "${SKIP_BENCH:-}" ]; then
    timeout -k 10 ${BENCH_LIMIT:-600} python3 -u bench.py --config "$c" ${BENCH_ARGS:-} > "$D/bench.log" 2>&1
    rc=$?; echo "[$c] bench rc=$rc: $(tail -c 300 "$D/bench.log" | tr -d '\n' | tail -c 200)"
    [ $rc = 0 ] || exit $rc
  fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- \
    python3 bench.py --config "$c" --steps 3 --warmup 1 --no-cpu-baseline --no-converge > "$D/trace.log" 2>&1
  rc=$?; echo "[$c] trace rc=$rc"; [ $rc = 0 ] || exit $rc
  if [ "${PMC:-1}" = 1 ]; then
    for p in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $p --kernel-trace --output-format csv -d "$D/$p" -o run -- \
        python3 bench.py --config "$c" --steps 1 --warmup 0 --no-cpu-baseline --no-converge > "$D/$p.log" 2>&1
      rc=$?; echo "[$c] $p rc=$rc"; [ $rc = 0 ] || exit $rc
    done
  fi
done
