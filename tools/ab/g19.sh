set -o pipefail
FILE=xt_kernels VARIANTS=b ROUNDS=2 bash tools/ab/run_ab.sh && FILE=xt_xcw VARIANTS=c ROUNDS=2 bash tools/ab/run_ab.sh
