#!/bin/bash
# run a subset of the GPU suite: TESTS="file::name ..." or -k expression in K
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-k}
timeout -k 10 ${LIMIT:-600} python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:-tests} ${K:+-k "$K"} > gpurun_out/${T}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${T}_tests.log; exit $rc
