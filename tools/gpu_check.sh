#!/bin/bash
# One GPU call: GPU parity tests, the default bench line, then a rocprofv3 kernel-trace pass.
set -euo pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-check}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
echo "pytest done"; tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.log" 2>&1
echo "bench done"; tail -1 "$OUT/bench.log"
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-converge > "$OUT/trace.log" 2>&1
  echo "trace done"
fi
