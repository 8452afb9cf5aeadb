#!/bin/bash
# rocprofv3 passes for the round-1 bench command (run on the GPU box from the repo root).
#   1) kernel trace + stats of the bench command
#   2) PMC FETCH_SIZE pass, 3) PMC WRITE_SIZE pass (separate passes, MI355X_MICROARCH.md HBM section)
set -euo pipefail
export TMPDIR=/tmp
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${PROF_TAG:-prof_r01}
mkdir -p "$OUT"
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline --no-converge"}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
echo "trace pass done"
PMC_ARGS=${PMC_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline --no-converge"}
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- python3 bench.py $PMC_ARGS > "$OUT/fetch.log" 2>&1
echo "fetch pass done"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- python3 bench.py $PMC_ARGS > "$OUT/write.log" 2>&1
echo "write pass done"
