set -o pipefail
FILE=xt_xcm VARIANTS="e f" ROUNDS=2 bash tools/ab/run_ab.sh && FILE=xt_xcw VARIANTS="g h" ROUNDS=2 bash tools/ab/run_ab.sh
