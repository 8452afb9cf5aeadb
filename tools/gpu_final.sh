#!/bin/bash
# round-end evidence in one call: the whole GPU suite, smoke(), the headline bench line
# (CPU baseline + Davidson convergence), rocprofv3 kernel stats and FETCH/WRITE passes
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-final}
timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > gpurun_out/${T}_pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
TAG=${T}_ev CONFIGS=${CONFIGS:-H} bash tools/evidence.sh
