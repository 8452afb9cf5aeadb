# SCF exchange from the orbital factors: device mean-field tests, then the porphyrin SCF time
set -o pipefail
mkdir -p gpurun_out/r06g22
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_frontend.py tests/test_gpu_molecule.py > gpurun_out/r06g22/pytest.log 2>&1 || { tail -30 gpurun_out/r06g22/pytest.log; exit 1; }
tail -2 gpurun_out/r06g22/pytest.log
timeout -k 10 400 python -u tools/molecule_run.py --molecule porphyrin --scf-only > gpurun_out/r06g22/porph.log 2>&1 || { tail -20 gpurun_out/r06g22/porph.log; exit 1; }
grep -E "^scf" gpurun_out/r06g22/porph.log
