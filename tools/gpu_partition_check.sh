#!/bin/bash
# GPU suite + a 2-rank rehearsal of the sharded bench on one GPU (gloo, ranks share the card).
set -uo pipefail
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-part}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --nao 400 --nc 39 --steps 3 --warmup 1 --no-cpu-baseline --no-converge > "$OUT/bench1.log" 2>&1
rc=$?; tail -1 "$OUT/bench1.log"; [ $rc = 0 ] || exit $rc
XT_BENCH_BACKEND=gloo timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --nao 400 --nc 39 --steps 3 --warmup 1 --converge > "$OUT/bench2.log" 2>&1
rc=$?; tail -1 "$OUT/bench2.log"; exit $rc
