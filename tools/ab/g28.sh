set -o pipefail
FILE=xt_gemm VARIANTS=b ROUNDS=2 bash tools/ab/run_ab.sh && FILE=xt_gemm VARIANTS=b ROUNDS=1 BENCH_ARGS="--config C4" bash tools/ab/run_ab.sh
