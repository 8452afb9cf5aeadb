set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest tests/test_gpu_qc.py tests/test_gpu_frontend.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06c/pytest_qc.log 2>&1 &&
timeout -k 10 900 python -u tools/molecule_run.py --molecule c60- --tol 1e-8 --out gpurun_out/r06c/r06_c60_xsf_tol1e-8.json > gpurun_out/r06c/c60_tol8.log 2>&1
