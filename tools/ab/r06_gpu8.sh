set -o pipefail
mkdir -p gpurun_out/r06g
timeout -k 10 900 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_qc.py tests/test_gpu_molecule.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r06g/pytest.log 2>&1 &&
timeout -k 10 600 python -u tools/molecule_run.py --molecule c60- --scf-only --out gpurun_out/r06g/c60_scf.json > gpurun_out/r06g/c60_scf.log 2>&1
