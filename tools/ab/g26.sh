set -o pipefail
FILE=xt_xcw VARIANTS=m ROUNDS=2 bash tools/ab/run_ab.sh || exit 1
cp tools/ab/xt_xcw_m.hip xtddft_amd/csrc/xt_xcw.hip; cp tools/ab/lib_m.so xtddft_amd/_lib/libxtddft_amd.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_variants.py tests/test_gpu_parity.py tests/test_gpu_molecule.py tests/test_gpu_configs.py > gpurun_out/g26_tests.log 2>&1; tail -3 gpurun_out/g26_tests.log
