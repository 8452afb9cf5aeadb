# round-6 final (a): the whole GPU suite and smoke() at HEAD
set -o pipefail
mkdir -p gpurun_out/r06fz
timeout -k 10 1080 python -u -m pytest -m gpu -x -q --timeout 900 --timeout-method thread tests > gpurun_out/r06fz/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06fz/pytest.log; exit 1; }
tail -2 gpurun_out/r06fz/pytest.log
timeout -k 10 100 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06fz/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r06fz/smoke.log; exit 1; }
tail -2 gpurun_out/r06fz/smoke.log
