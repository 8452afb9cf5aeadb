set -o pipefail
FILE=xt_ctx BENCH_ARGS="--config C2" ROUNDS=1 bash tools/ab/run_ab.sh && FILE=xt_ctx BENCH_ARGS="--config C5" ROUNDS=1 bash tools/ab/run_ab.sh
