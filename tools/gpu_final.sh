#!/bin/bash
# Round evidence in one GPU call: smoke, the GPU suite, the headline evidence
# (bench line + rocprof trace + PMC passes, tools/evidence.sh) and the integral timings.
set -uo pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-final}
mkdir -p "$OUT"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc = 0 ] || exit $rc
TAG=${TAG:-final}/ev CONFIGS="${CONFIGS:-H}" bash tools/evidence.sh || exit 1
timeout -k 10 300 python -u tools/int_bench.py 1 2 4 8 > "$OUT/int_bench.jsonl" 2>&1
rc=$?; cat "$OUT/int_bench.jsonl" | tail -4; exit $rc
