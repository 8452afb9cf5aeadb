set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_parity.py > gpurun_out/g24_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/g24_tests.log; exit 1; }
tail -1 gpurun_out/g24_tests.log
FILE=xt_xcm VARIANTS="i j k" ROUNDS=2 bash tools/ab/run_ab.sh
