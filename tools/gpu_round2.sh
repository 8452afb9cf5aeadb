#!/bin/bash
# Round-2 GPU check: the -m gpu suite, the headline bench, and the self-launched
# 2-rank bench rehearsed over gloo on the one GPU.  Each step under its own limit.
set -o pipefail
OUT=gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
  tail -c 600 "$OUT/bench.log"
  XT_BENCH_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 2 --warmup 1 --nao 400 --nclosed 39 > "$OUT/bench_gpus2.log" 2>&1 || { echo "bench2 failed"; tail -20 "$OUT/bench_gpus2.log"; exit 1; }
  tail -c 400 "$OUT/bench_gpus2.log"
fi
