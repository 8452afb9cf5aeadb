# blocked in-batch Cholesky pivoting: front-end tests, then the porphyrin front end (SCF only)
set -o pipefail
mkdir -p gpurun_out/r06g11
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frontend.py > gpurun_out/r06g11/pytest.log 2>&1 || { tail -30 gpurun_out/r06g11/pytest.log; exit 1; }
tail -2 gpurun_out/r06g11/pytest.log
timeout -k 10 600 python -u tools/molecule_run.py --molecule porphyrin --scf-only --out gpurun_out/r06g11/porph.json > gpurun_out/r06g11/porph.log 2>&1 || { tail -20 gpurun_out/r06g11/porph.log; exit 1; }
grep -E "chol|scf|build" gpurun_out/r06g11/porph.log | tail -8
